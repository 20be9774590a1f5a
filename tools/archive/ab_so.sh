# A/B two builds of the native module in ONE GPU call (box-to-box variance is ~5 %):
# put them at tmp_so/old.so and tmp_so/new.so, then: gpurun -- bash tools/ab_so.sh
# Two rounds of MNIST (8 x 64), Otto (8 x 128) and Wide (1 x 1024); gpurun_out/ab.log.
SO=elephas_amd/_C.cpython-310-x86_64-linux-gnu.so
mkdir -p gpurun_out
for round in 1 2; do for v in old new; do cp tmp_so/$v.so $SO; for m in ${AB_MODELS:-mnist otto wide}; do
  extra="--steps 1500 --warmup 150"
  [ $m = otto ] && extra="--batch 128 --steps 1500 --warmup 150"
  [ $m = wide ] && extra="--workers-per-gpu 1 --batch 1024 --steps 100 --warmup 10"
  timeout -k 10 200 python bench.py --model $m $extra 2>/dev/null | tail -n1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$round $v $m', d['ms_per_step'])" >> gpurun_out/ab.log || exit 1
done; done; done
cat gpurun_out/ab.log
