#!/bin/bash
# group-accumulator add at B1 without a return value, read back by the look-back (OPT 1073741824)
set -u
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:1073742096,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:1073742864,v4:32:0:1024:36:1:280,v4:32:0:1024:36:1:1073742104,v4:32:0:768:64:1:1048,v4:32:0:768:64:1:1073742872 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:1073742864,v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:1073742096 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --check --variants v4:32:1:768:40:1:1040,v4:32:1:768:40:1:1073742864,v4:64:0:768:44:1:1040,v4:64:0:768:44:1:1073742864 || exit $?
