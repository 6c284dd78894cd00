set -e
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none > gpurun_out/gc_off_$i.log 2>&1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-events none --gc-in-steps > gpurun_out/gc_on_$i.log 2>&1
done
for i in 1 2 3; do echo "gc off $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gc_off_$i.log | head -1) on $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gc_on_$i.log | head -1)"; done
