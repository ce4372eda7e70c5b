#!/bin/bash
# store-pattern emulation map: run length (36K / 48K / 72K tiles), alignment (mode 1 vs 3),
# XCD-local tiles (mode 2 / 5), store policy (x1 nt, x2 sc1) at 2^28 and 2^30
set -u
E=1024:36:0:150000,1024:36:1:150000,1024:36:3:150000,1024:36:2:150000,1024:36:5:150000,1024:36:11:150000,1024:36:13:150000,1024:36:21:150000,1024:36:23:150000,1024:48:0:150000,1024:48:1:150000,1024:48:3:150000,1024:48:5:150000,1024:72:0:150000,1024:72:1:150000,1024:72:3:150000,1024:72:5:150000
python -u tools/lab2.py --n 268435456 --rounds 5 --variants v4:32:0:1024:36:1:272 --emu $E || exit $?
python -u tools/lab2.py --n 1073741824 --rounds 3 --variants v4:32:0:1024:36:1:272 --emu $E || exit $?
