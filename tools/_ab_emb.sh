set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "feat_embed" > gpurun_out/t_emb.log 2>&1 || (tail -n 30 gpurun_out/t_emb.log; exit 1)
tail -n 1 gpurun_out/t_emb.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullshape.py > gpurun_out/t_par.log 2>&1 || (tail -n 30 gpurun_out/t_par.log; exit 1)
tail -n 1 gpurun_out/t_par.log
for i in 1 2 3; do
  CTR_LIB_PATH=$PWD/exp/lib_embold.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > gpurun_out/ab_base_$i.log 2>&1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > gpurun_out/ab_exp_$i.log 2>&1
done
for i in 1 2 3; do echo "old $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_base_$i.log | head -1) new $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_exp_$i.log | head -1)"; done
