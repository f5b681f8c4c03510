#!/bin/bash
# Vector stride vs HBM mapping: vs = align(2^26 elements) + P ("plane-like" low address
# bits, as the plane-interleaved layout of tools/bw_probe5) vs the default 4 KiB pad.
set -e
O=gpurun_out/pad2; mkdir -p $O
timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/default.json
NLS_VEC_PAD=66846720 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/planeish.json
NLS_VEC_PAD=66715648 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/halfplane.json
NLS_VEC_PAD=67108864 timeout -k 10 200 python tools/perj.py nlse3d_512 > $O/plus1g.json
