#!/bin/bash
set -u
for a in "--steps 200" "--model qgnni --code toric_5 --steps 200"; do bash tools/ab_quick.sh new2 "$a" 2 || exit $?; done
