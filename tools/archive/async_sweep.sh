set -u
O=gpurun_out/async_epoch.log
for args in "--mode asynchronous --frequency epoch" "--mode asynchronous --frequency epoch --async-groups 2" "--mode asynchronous --frequency epoch --async-groups 1" "--mode hogwild --frequency epoch" "--mode asynchronous --frequency batch"; do
  echo "== $args" >> $O
  timeout -k 10 200 python bench.py --steps 1000 --warmup 100 $args >> $O 2>&1 || exit 1
done
