#!/opt/conda/bin/python3.9
"""Generate tests/golden/quant.npz + quant.json (run in the build container only).

Interpreter: /opt/conda/bin/python3.9 with scikit-learn 0.24.2 and Pillow 8.4.0.  The reference
pins scikit-learn 0.20.3 and pillow 6.2.1 (requirements.txt:132,161); MiniBatchKMeans in 0.20 and
0.24 is the same pre-1.0 algorithm (k-means++ init over init_size samples, n_init=3, batch_size
100, EWA-inertia early stopping, labels_ from a final full assignment), and Pillow's
ImageEnhance.Brightness is the same ImagingBlend against a black image in both.

quant (lib/model/test.py:592-765, lib/roi_data_layer/minibatch.py:492-667):
    lab = cv2.cvtColor(img, COLOR_BGR2LAB); clt = MiniBatchKMeans(n_clusters=k)
    labels = clt.fit_predict(lab.reshape(-1, 3)); quant = clt.cluster_centers_.astype('uint8')[labels]
cv2 is not importable here, so `lab` comes from the oracle restatement (oracle/cvlab.py, parity
vs cv2 unpinned); what IS pinned by these fixtures is sklearn's fit on that input: the fitted
centres, the labels fit_predict returns and the inertia.  The reference never seeds
MiniBatchKMeans; the fixtures use random_state=0 so they are reproducible.

shader (lib/model/test.py:1595-1601):
    np.array(ImageEnhance.Brightness(Image.open(path)).enhance(3))   (RGB array)
with real Pillow on the RGB view of the BGR inputs.

  /opt/conda/bin/python3.9 tests/golden/make_quant_fixtures.py
"""
import json
import sys
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent
ROOT = OUT.parent.parent
DEMO = Path("/root/reference/data/demo")
sys.path.insert(0, str(ROOT))

from oracle import cvlab  # noqa: E402


def make_img(h, w, seed):
    """integer-only synthetic BGR image: a few colour regions plus noise (k-means has structure
    to find)."""
    rs = np.random.RandomState(seed)
    y, x = np.mgrid[0:h, 0:w]
    region = ((x * 3 // w) + 3 * (y * 2 // h)) % 6
    palette = rs.randint(20, 236, size=(6, 3))
    img = palette[region] + rs.randint(-25, 26, size=(h, w, 3))
    return np.clip(img, 0, 255).astype(np.uint8)


def demo_crop(name, y0, x0, h, w):
    from PIL import Image
    rgb = np.asarray(Image.open(DEMO / name).convert("RGB"))
    return np.ascontiguousarray(rgb[y0:y0 + h, x0:x0 + w, ::-1])


def main():
    import PIL
    import sklearn
    from PIL import Image, ImageEnhance
    from sklearn.cluster import MiniBatchKMeans

    inputs = {
        "syn64": make_img(64, 96, 5),
        "syn120": make_img(120, 200, 6),
        "demo456": demo_crop("000456.jpg", 100, 150, 120, 200),
        "demo1763": demo_crop("001763.jpg", 60, 100, 120, 200),
    }
    arrays = {f"in_{k}": v for k, v in inputs.items()}
    meta = {"generator": "tests/golden/make_quant_fixtures.py",
            "versions": {"sklearn": sklearn.__version__, "PIL": PIL.__version__,
                         "numpy": np.__version__},
            "quant": [], "shader": []}
    for name, img in inputs.items():
        lab = cvlab.bgr2lab(img)
        X = lab.reshape(-1, 3)
        for k in (3, 7, 10):
            clt = MiniBatchKMeans(n_clusters=k, random_state=0)
            labels = clt.fit_predict(X)
            key = f"{name}_k{k}"
            arrays[f"centers_{key}"] = clt.cluster_centers_.astype(np.float64)
            arrays[f"labels_{key}"] = labels.astype(np.uint8).reshape(img.shape[:2])
            meta["quant"].append({"case": key, "input": name, "k": k,
                                  "inertia": float(clt.inertia_)})
        rgb = np.ascontiguousarray(img[..., ::-1])
        out = np.asarray(ImageEnhance.Brightness(Image.fromarray(rgb)).enhance(3))
        arrays[f"shader_{name}"] = out.astype(np.uint8)
        meta["shader"].append({"input": name, "factor": 3})
    np.savez_compressed(OUT / "quant.npz", **arrays)
    (OUT / "quant.json").write_text(json.dumps(meta, indent=1) + "\n")
    print("wrote", OUT / "quant.npz", sum(a.nbytes for a in arrays.values()), "bytes raw")


if __name__ == "__main__":
    main()
