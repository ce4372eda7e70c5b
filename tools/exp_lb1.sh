#!/bin/bash
# look-back window / group size / issue point at 2^28 (ns) and 2^24 (C2 size; 8- and 4-bit)
set -u
for lib in "" gw16 g16; do
  echo "#### lib=$lib"
  python -u tools/lab2.py ${lib:+--lib $lib} --n 268435456 --rounds 5 \
    --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:1024,v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:256 || exit $?
  python -u tools/lab2.py ${lib:+--lib $lib} --n 16777216 --rounds 7 --check \
    --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:256,v6:32:0:1024:36:1:272:256,r6:32:0:1024:32:1:0:256,r6:32:0:1024:32:1:8:256 || exit $?
done
