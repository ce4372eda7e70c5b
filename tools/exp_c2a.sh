#!/bin/bash
# C2 (2^24 u32, 4-bit): ballot-match ranking vs lane-ordered LDS atomics in the persistent pass
set -u
python -u tools/lab2.py --n 16777216 --rounds 9 --check \
  --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:512:256,r6:32:0:1024:32:1:528:256,r6:32:0:1024:32:1:8:256,r6:32:0:1024:32:1:520:256 || exit $?
