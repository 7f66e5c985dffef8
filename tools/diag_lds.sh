#!/bin/bash
# LDS bank-conflict attribution of the headline kernel (decode_resident_kernel, BCH CGNNI): builds
# whose LDS accesses of one kind are replaced by lane-linear, conflict-free addresses (outputs
# WRONG: timing and counters only) against the real kernel, kernel time (two runs each) and the
# LDS counters of one PMC pass.  Build the variants first:
#   tools/build_variant.sh diagtv  -DGNND_DIAG_TV_LINEAR    (check step's T_v gathers)
#   tools/build_variant.sh diagmsg -DGNND_DIAG_MSG_LINEAR   (check step's message writes)
#   tools/build_variant.sh diagvar -DGNND_DIAG_VAR_LINEAR   (variable step's run reads, T writes)
#   tools/build_variant.sh diagall "-DGNND_DIAG_TV_LINEAR -DGNND_DIAG_MSG_LINEAR -DGNND_DIAG_VAR_LINEAR"
set -u
mkdir -p gpurun_out/diag
for rep in 1 2; do
  for lib in base diagtv diagmsg diagvar diagall; do
    if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
    timeout -k 10 120 python bench.py --steps 100 --warmup 3 --configs off --cpu-seconds 0 > gpurun_out/diag/b.log 2>&1 || exit $?
    tail -n 1 gpurun_out/diag/b.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib', round(j['value']), round(j['roofline']['kernel_ms'],4))"
  done
done
for lib in base diagtv diagmsg diagvar diagall; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/diag/pmc_$lib -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --configs off --cpu-seconds 0 > gpurun_out/diag/pmc_$lib.log 2>&1 || exit $?
  python tools/pmc_kernels.py gpurun_out/diag/pmc_$lib gpurun_out/diag/pmc_$lib.json decode_resident > /dev/null
  python -c "
import json; d=json.load(open('gpurun_out/diag/pmc_$lib.json'))
for k,v in d.items():
    print('$lib', 'conflict/ldsactive', round(v['SQ_LDS_BANK_CONFLICT']/v['SQ_LDS_IDX_ACTIVE'],3), 'wait_any', round(v['SQ_WAIT_ANY']/v['SQ_WAVE_CYCLES'],3), 'lds_active/gui', round(v['SQ_LDS_IDX_ACTIVE']/v['GRBM_GUI_ACTIVE'],3))"
done
