set -o pipefail
mkdir -p gpurun_out/tr1
export MASTER_ADDR=127.0.0.1
echo "=== torchrun decode $(date +%T)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/tr1/torchrun_decode.log 2>&1 && tail -c 600 gpurun_out/tr1/torchrun_decode.log &&
echo "=== torchrun train $(date +%T)" &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --mode train --steps 20 --warmup 3 > gpurun_out/tr1/torchrun_train.log 2>&1 && tail -c 400 gpurun_out/tr1/torchrun_train.log &&
echo "=== default bench $(date +%T)" &&
( time timeout -k 10 400 python bench.py > gpurun_out/tr1/default_bench.log 2>&1 ) 2> gpurun_out/tr1/default_bench.time && cat gpurun_out/tr1/default_bench.time && tail -c 300 gpurun_out/tr1/default_bench.log &&
echo "=== done $(date +%T)"
