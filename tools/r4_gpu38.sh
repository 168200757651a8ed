# round 4: N=2 launch rehearsal on the one-GPU box (both ranks share the GPU; checks the launch, barrier and reduction)
(while sleep 50; do date >> gpurun_out/tick.log; done) &
TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/r4_bench_n2.json 2> gpurun_out/r4_bench_n2.err
