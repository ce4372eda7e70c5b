#!/bin/bash
# C2 pass: what the look-back costs (OPT 64 estimates the prefixes: wrong output, timing only)
# and the wide look-back, with stamps
set -u
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 15 --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:64:256,r6:32:0:1024:32:1:2097152:256,r6:32:0:1024:32:1:8:256,r6:32:0:1024:32:1:72:256,r6:32:0:1024:32:1:2097160:256 || exit $?
