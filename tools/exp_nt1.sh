#!/bin/bash
# tile = blockIdx.x (OPT 4194304, no ticket round trip) vs ticketed v4: big / XL tiles at 2^28 and
# 2^30, u32 pairs and u64 keys at 2^28; stamps of both
set -u
V28=v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:4194576,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:4195344
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants $V28,v4:32:0:1024:36:1:280,v4:32:0:1024:36:1:4194584,v4:32:0:768:64:1:1048,v4:32:0:768:64:1:4195352 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants $V28 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --check --variants v4:32:1:768:40:1:1040,v4:32:1:768:40:1:4195344,v4:64:0:768:44:1:1040,v4:64:0:768:44:1:4195344 || exit $?
# persistent without prefetch (OPT 8388608): next ticket drawn during the ranking, loads after the tile
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:8388880:256,v4:32:0:768:64:1:1040,v6:32:0:768:64:1:8389648:256,v6:32:0:1024:36:1:8388888:256,v6:32:0:768:64:1:8389656:256 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v6:32:0:768:64:1:8389648:256,v4:32:0:768:64:1:4195344 || exit $?
