#!/bin/bash
# C2 (2^24 keys, 4-bit digits, persistent pass): occupancy / tile shapes, and the digit wave
# kept out of the prefetch (OPT 524288, its look-back polls then do not wait behind the loads)
set -u
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 15 --check --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:524288:256,r6:32:0:512:32:2:0:512,r6:32:0:512:32:2:524288:512,r6:32:0:256:32:4:0:1024,r6:32:0:1024:16:1:0:256,r6:32:0:512:16:2:0:512,r6:32:0:1024:32:1:8:256,r6:32:0:1024:32:1:524296:256,r6:32:0:512:32:2:8:512 || exit $?
