#!/bin/bash
# destination-aligned stores (OPT 65536) vs the library pass: 2^28 and 2^30 u32 keys, checks
set -u
V=v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:65808,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:66576
python -u tools/lab2.py --n 268435456 --rounds 7 --check \
  --variants $V,v4:32:0:1024:36:1:65816,v4:32:0:768:64:1:66584 || exit $?
python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:66576,v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:65808 || exit $?
python -u tools/lab2.py --n 16777219 --rounds 2 --check \
  --variants v4:32:1:1024:17:1:65808,v4:32:1:768:40:1:66576,v4:64:0:1024:17:1:65808,v4:64:0:768:44:1:66576,v6:32:0:1024:36:1:65792:256,v4:32:0:768:64:1:66576 || exit $?
