# A/B an environment knob of ONE build in one GPU call (box-to-box variance is ~5 %):
#   gpurun -- bash tools/ab_env.sh ELEPHAS_AMD_KSPEC 0 1
# Two rounds of MNIST (8 x 64) and Otto (8 x 128); results in gpurun_out/ab_env.log.
KNOB=$1; A=$2; B=$3
mkdir -p gpurun_out
for round in 1 2; do for v in $A $B; do for m in mnist otto; do
  extra=""; [ $m = otto ] && extra="--batch 128"
  env $KNOB=$v timeout -k 10 200 python bench.py --model $m $extra --steps 1500 --warmup 150 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $KNOB=$v $m', d['ms_per_step'])" >> gpurun_out/ab_env.log || exit 1
done; done; done
cat gpurun_out/ab_env.log
