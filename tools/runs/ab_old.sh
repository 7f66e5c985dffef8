#!/bin/bash
set -u
for a in "--model qgnni --code toric_5 --steps 200" "--steps 200" "--code ldpc_648_324 --batch 131072 --steps 30" "--model qbp --code toric_5 --steps 200"; do bash tools/ab_quick.sh old "$a" 2 || exit $?; done
