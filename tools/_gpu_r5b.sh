set -e
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lazy.py -k "tiny_block or tiny_concat" > gpurun_out/t_block.log 2>&1 || (tail -n 40 gpurun_out/t_block.log; exit 1)
tail -n 1 gpurun_out/t_block.log
bash tools/_ab_cfg4.sh aw4
