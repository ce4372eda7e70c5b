#!/bin/bash
# speculative tile loads (OPT 131072) vs the library pass at 2^28 and 2^30; ticket latency stamps
set -u
python -u tools/lab2.py --n 268435456 --rounds 7 --check \
  --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:131344,v4:32:0:1024:36:1:280,v4:32:0:1024:36:1:131352 || exit $?
python -u tools/lab2.py --n 1073741824 --rounds 5 \
  --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:132112,v4:32:0:768:64:1:1048,v4:32:0:768:64:1:132120 || exit $?
python -u tools/lab2.py --n 16777219 --rounds 2 --check \
  --variants v4:32:1:1024:17:1:131344,v4:64:0:1024:17:1:131344,v4:32:0:768:64:1:132112 || exit $?
