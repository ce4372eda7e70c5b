#!/bin/bash
# ns (2^28 u32 keys) pass experiments: phase stamps of the big and XL tiles, store-pattern
# emulation and the copy / read ceilings at the same size.
set -u
python -u tools/lab2.py --n 268435456 --rounds 5 \
  --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:280,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:1048 \
  --emu 1024:36:0:150000,1024:36:1:150000,1024:36:3:150000 --copy
