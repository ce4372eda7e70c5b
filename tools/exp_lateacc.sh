#!/bin/bash
# group-accumulator add issued at the look-back's finish (OPT 536870912) instead of at B1
set -u
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 9 --check --variants v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:536871184,v4:32:0:768:64:1:1040,v4:32:0:768:64:1:536871952,v4:32:0:1024:36:1:280,v4:32:0:1024:36:1:536871192,v4:32:0:768:64:1:1048,v4:32:0:768:64:1:536871960 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 1073741824 --rounds 5 --variants v4:32:0:768:64:1:1040,v4:32:0:768:64:1:536871952,v4:32:0:1024:36:1:272,v4:32:0:1024:36:1:536871184 || exit $?
timeout -k 10 240 python -u tools/lab2.py --n 268435456 --rounds 7 --check --variants v4:32:1:768:40:1:1040,v4:32:1:768:40:1:536871952,v4:64:0:768:44:1:1040,v4:64:0:768:44:1:536871952 || exit $?
