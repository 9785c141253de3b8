#!/bin/bash
# quick GPU loop: golden + subsampled parity grids, then HIP-event timing of fwd/bwd at cfg3
set -o pipefail
FA2_GRID_STRIDE=${STRIDE:-9} timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider 2>&1 | tail -2 || exit 1
timeout -k 10 120 python scripts/time_fwd.py || exit 1
if [ -n "$NONCAUSAL" ]; then CAUSAL=0 timeout -k 10 120 python scripts/time_fwd.py || exit 1; fi
