cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_v19; mkdir -p $O
INSFM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config 2 --steps 5 --warmup 2 --no-cpu --no-solve > $O/gloo2_config2.json 2> $O/gloo2_config2.err || exit 1
timeout -k 10 200 python -u bench.py --config 2 --steps 5 --warmup 2 --no-cpu --no-solve > $O/n1_config2.json 2> $O/n1_config2.err || exit 1
