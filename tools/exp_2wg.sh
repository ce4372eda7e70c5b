#!/bin/bash
# two workgroups per CU (MINW 2, 512 threads): the LDS phases of one tile overlap the HBM phases
# of the other, at half the tile (more digit-run boundaries).  2^28 and 2^30 u32 keys.
set -u
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants v4:32:0:1024:36:1:272,v4:32:0:512:36:2:272,v4:32:0:512:32:2:272,v4:32:0:512:48:2:1040,v4:32:0:512:56:2:1040,v4:32:0:512:64:2:1040,v4:32:0:768:64:1:1040,v4:32:0:512:36:2:280 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v4:32:0:512:36:2:272,v4:32:0:512:48:2:1040,v4:32:0:512:56:2:1040 || exit $?
