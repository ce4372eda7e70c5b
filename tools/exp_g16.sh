#!/bin/bash
# 16-lane-group counter sets (OPT 67108864): C2's 4-bit persistent pass (and with stamps), and
# the 8-bit big / XL passes with 32-bit counters (G16 excludes the 16-bit ones)
set -u
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 15 --check --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:67108864:256,r6:32:0:1024:32:1:8:256,r6:32:0:1024:32:1:67108872:256,r6:32:0:1024:32:1:67108880:256 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 16777219 --rounds 3 --check --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:67108864:256 || exit $?
