set -e
mkdir -p gpurun_out/sweep
F="--no-cpu-baseline --no-spmv --no-be --no-c2 --no-3d --steps 40"
for cfg in "MMX_PROX_BLOCK=128" "MMX_PROX_BLOCK=64" "MMX_PROX_BLOCK=256" "MMX_XCD_MAP=0" "MMX_GRAD_CACHE=0" "MMX_PROX_BLOCK=128"; do
  n=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 120 python bench.py $F > gpurun_out/sweep/$n.json 2> gpurun_out/sweep/$n.err
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/sweep/$n.json'));print(d['value'],d['kernels'])")"
done
