#!/bin/bash
# persistent pass with split prefetch (OPT 524288) vs v4 at 2^28 / 2^30 / 2^27 / 2^26
set -u
python -u tools/lab2.py --n 268435456 --rounds 7 --check \
  --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:272:256,v6:32:0:1024:36:1:524560:256,v6:32:0:1024:36:1:524568:256,v6:32:0:1024:36:1:524560:512 || exit $?
python -u tools/lab2.py --n 1073741824 --rounds 5 \
  --variants v4:32:0:768:64:1:1040,v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:524560:256 || exit $?
python -u tools/lab2.py --n 134217728 --rounds 7 \
  --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:272:256,v6:32:0:1024:36:1:524560:256 || exit $?
python -u tools/lab2.py --n 16777219 --rounds 3 --check \
  --variants v6:32:1:1024:17:1:524560:256,v6:64:0:1024:17:1:524560:256,v6:32:0:1024:36:1:524560:256 || exit $?
