#!/bin/bash
# C2 pass (2^24 u32, 4-bit, persistent) with XCD ranges (one pass, lab-computed per-range histograms)
set -u
python -u tools/lab2.py --n 16777216 --rounds 9 --check \
  --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:1048576:256,r6:32:0:1024:32:1:8:256,r6:32:0:1024:32:1:1048584:256 || exit $?
