#!/bin/bash
# A/B of environment knobs on the C3 bench: scripts/ab_env.sh "VAR=a" "VAR=b" ...  (one bench per setting,
# each under its own time limit; stops at the first fault/timeout).  Output: gpurun_out/ab.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for setting in "$@"; do
  env $setting timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-15} --warmup 3 ${AB_ARGS:-} > gpurun_out/ab_run.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$setting rc=$rc" >> gpurun_out/ab.txt; tail -5 gpurun_out/ab_run.log >> gpurun_out/ab.txt; exit $rc; fi
  python - "$setting" >> gpurun_out/ab.txt <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab_run.log") if l.startswith("{")][-1]
d = json.loads(line)
ph = " ".join(f"{k}={v:.3f}" for k, v in d.get("phases_ms", {}).items())
print(f"{sys.argv[1]:40s} {d['value']:8.2f} steps/s  {d['ms_per_step']:.3f} ms  {ph}")
PY
done
