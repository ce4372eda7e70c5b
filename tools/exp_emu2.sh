#!/bin/bash
# destination-aligned chunk stores of misaligned runs (emu mode 8), default vs nontemporal
# interiors, against the plain misaligned sweep (mode 3) and aligned runs (mode 1)
set -u
E=1024:36:0:150000,1024:36:1:150000,1024:36:3:150000,1024:36:8:150000,1024:36:38:150000,1024:36:11:150000,1024:36:31:150000,1024:48:3:150000,1024:48:8:150000,1024:48:38:150000
python -u tools/lab2.py --n 268435456 --rounds 5 --variants v4:32:0:1024:36:1:272 --emu $E || exit $?
python -u tools/lab2.py --n 1073741824 --rounds 3 --variants v4:32:0:768:64:1:1040 --emu $E || exit $?
