cd $GRAFT_REPO_ROOT
for K in 16 12 14 20 16 12 14; do
  timeout -k 10 100 python bench.py --no-cpu --no-solve --cluster-size $K > gpurun_out/k_$K.log 2>&1 || exit 1
  echo "K=$K $(grep -o '"value": [0-9.]*' gpurun_out/k_$K.log | head -1) $(grep -o '"pcg_iters": \[[^]]*\]' gpurun_out/k_$K.log) $(grep -o '"cg_iterations": [0-9.]*' gpurun_out/k_$K.log)"
done
