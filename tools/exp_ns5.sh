#!/bin/bash
# persistent pass (ticket + next tile prefetched) vs one tile per workgroup at 2^28 / 2^30
set -u
python -u tools/lab2.py --n 268435456 --rounds 7 --check \
  --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:272:256,v6:32:0:1024:36:1:262416:256,v4:32:0:1024:36:1:280,v6:32:0:1024:36:1:280:256,v6:32:0:1024:36:1:262424:256 || exit $?
python -u tools/lab2.py --n 1073741824 --rounds 5 \
  --variants v4:32:0:1024:36:1:272,v6:32:0:1024:36:1:272:256,v6:32:0:1024:36:1:262416:256 || exit $?
