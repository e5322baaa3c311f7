cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pad
for pad in 0 32 0 32 64 128; do
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --log-pad $pad > gpurun_out/pad/p$pad.json 2>gpurun_out/pad/p$pad.err || exit 1
echo "pad $pad: $(grep 'per step' gpurun_out/pad/p$pad.err)"
done
