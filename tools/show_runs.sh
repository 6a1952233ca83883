#!/bin/bash
# Summaries of tools/gpu_g2.sh's bench and stamp logs (build container side).
cd "$(dirname "$0")/.." || exit 2
for f in b_cabf b_vbpff b_caff; do
  [ -f gpurun_out/$f.log ] || continue
  tail -1 gpurun_out/$f.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{})
print('$f', round(d['ms_per_step'],4), 'parity', d.get('parity'), 'walk', r.get('walk_ms_per_step') and round(r['walk_ms_per_step'],4), 'cyc/task', r.get('cycles_per_task') and round(r['cycles_per_task']), {k: round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})"
done
grep -h "walk \|pass\|search\|batches\|single\|bulk" gpurun_out/st_*.log 2>/dev/null
