cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ord
for rep in 1 2; do for o in ${ORDERS:-natural lpt-xcd random}; do
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --group-order $o > gpurun_out/ord/$o$rep.json 2>gpurun_out/ord/$o$rep.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ord/$o$rep.json')); r=d['roofline']; print('$o', round(r['kernel_ms_mean']*1e3,1), round(r['kernel_ms_min']*1e3,1), round(r['frac'],3))"
done; done
