#!/bin/bash
# round 6: counters of the two-read Haar-3 path (wavelet_haar3, cfg5): kernel trace + FETCH / WRITE
# / two SQ groups, folded by tools/pmc_r04.py into profiles/r06/pmc
set -u
bash tools/pmc_r04.sh r06k wavelet_haar3 cfg5 || exit 1
