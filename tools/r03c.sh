set -u
OUT=gpurun_out/r03c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/list_avail.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_at_size.py -k "split or unit" -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
for b in 16 128 1024; do timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b$b.log 2>&1 || exit 1; grep '^{' $OUT/b$b.log | tail -1 >> $OUT/curve.jsonl; done
for us in 4 2 1; do GNND_V24_SPLIT=$us timeout -k 10 200 python bench.py --mode train --batch 128 --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/us$us.log 2>&1 || exit 1; grep '^{' $OUT/us$us.log | tail -1 >> $OUT/curve_us.jsonl; done
bash tools/pmc_train.sh $OUT/pmc128 --batch 128 > $OUT/pmc128.log 2>&1 || { tail $OUT/pmc128.log; exit 1; }
echo done
