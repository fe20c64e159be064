# Portions of this file (prepare_roidb's body) follow Fast R-CNN's
#   lib/roi_data_layer/roidb.py -- Fast R-CNN, Copyright (c) 2015 Microsoft,
#   Licensed under The MIT License, written by Ross Girshick.
# The drop-in keeps that function's behaviour line for line so callers see identical entries.
"""Drop-in for lib/roi_data_layer/roidb.py:prepare_roidb(imdb, noise) (19-50): the step that
stamps the `--noise` spec on every roidb entry (roidb.py:50), i.e. the plugin surface on the
training side.  The derived-overlap fields are kept so get_minibatch's consumers see the same
entries; dataset I/O itself stays with the caller's imdb (out of scope)."""
from __future__ import annotations

import numpy as np


def prepare_roidb(imdb, noise):
    roidb = imdb.roidb
    if not imdb.name.startswith("coco"):
        from PIL import Image
        sizes = [Image.open(imdb.image_path_at(i)).size for i in range(imdb.num_images)]
    for i in range(len(imdb.image_index)):
        roidb[i]["image"] = imdb.image_path_at(i)
        roidb[i]["index"] = i
        if not imdb.name.startswith("coco"):
            roidb[i]["width"] = sizes[i][0]
            roidb[i]["height"] = sizes[i][1]
        gt_overlaps = roidb[i]["gt_overlaps"]
        if hasattr(gt_overlaps, "toarray"):
            gt_overlaps = gt_overlaps.toarray()
        gt_overlaps = np.asarray(gt_overlaps)
        max_overlaps = gt_overlaps.max(axis=1)
        max_classes = gt_overlaps.argmax(axis=1)
        roidb[i]["max_classes"] = max_classes
        roidb[i]["max_overlaps"] = max_overlaps
        zero_inds = np.where(max_overlaps == 0)[0]
        assert all(max_classes[zero_inds] == 0)
        nonzero_inds = np.where(max_overlaps > 0)[0]
        assert all(max_classes[nonzero_inds] != 0)
        roidb[i]["noise_type"] = noise
