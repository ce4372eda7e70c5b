#!/bin/bash
# persistent pass without prefetch (OPT 8388608), with and without draining the tile's stores
# before the next tile's loads (OPT 268435456), against the one-tile-per-workgroup v4
set -u
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:8388880:256,v6:32:0:1024:36:1:277086480:256,v4:32:0:768:64:1:1040,v6:32:0:768:64:1:277087248:256,v6:32:0:1024:36:1:8388888:256,v6:32:0:1024:36:1:277086488:256 || exit $?
