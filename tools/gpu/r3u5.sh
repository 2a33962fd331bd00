# Whole -m gpu suite + smoke with the unit K2 kernel, then the K2 choice per
# config: unit forced vs the 16-bit rows (swar16) on cfg3 / cfg5 / cfg2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3u5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for p in cfg3 cfg5 cfg2; do
  for i in 1 2; do
    for v in unit swar16; do
      GHOSTM_K2=$v timeout -k 10 300 python3 bench.py --preset $p --steps 5 --warmup 1 --no-cpu --no-e2e \
        --workdir /tmp/ghostm_ab_$p > $O/${p}_${v}_$i.log 2>&1 || exit $?
    done
  done
done
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "cfg*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = {k: round(v * 1e3, 2) for k, v in d["stages_s_per_step"].items() if k in ("total", "score_device")}
            print(os.path.basename(f), round(d["ms_per_step"], 2), st, d.get("full_output_matches_reference"))
PY
