cd ${GRAFT_REPO_ROOT:-$(pwd)}
for s in 1 2 4 7; do
  echo "== RC_SPLIT=$s"
  ELEPHAS_AMD_RC_SPLIT=$s timeout -k 10 120 python tools/stamps.py 8 mnist 64 float32 2>/dev/null | grep -E "row chain|^launch 0|^launch 2"
  ELEPHAS_AMD_RC_SPLIT=$s timeout -k 10 120 python bench.py --steps 2000 --warmup 200 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('us/step', d['ms_per_step']*1000)"
done
