#!/bin/bash
# pass store policy: default / all nontemporal (OPT 16777216) / nontemporal for the lines wholly
# inside a tile's digit run (OPT 33554432): big + XL u32 keys at 2^28 and 2^30, u32 pairs and u64
# keys at 2^28, the C2 4-bit persistent pass at 2^24 (single-launch times include the kernel's
# end-of-kernel L2 write-back)
set -u
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:16777488,v4:32:0:1024:36:1:33554704,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:16778256,v4:32:0:768:64:1:33555472 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:16778256,v4:32:0:768:64:1:33555472 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --check --variants v4:32:1:768:40:1:1040,v4:32:1:768:40:1:16778256,v4:32:1:768:40:1:33555472,v4:64:0:768:44:1:1040,v4:64:0:768:44:1:16778256,v4:64:0:768:44:1:33555472 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 16777216 --rounds 15 --check --variants r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:16777216:256,r6:32:0:1024:32:1:33554432:256 || exit $?
