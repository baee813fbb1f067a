#!/bin/bash
# Summarise gpurun_out/ after tools/gpu_check.sh
tail -1 gpurun_out/pytest_gpu.log 2>/dev/null
for f in gpurun_out/bench*.json; do
  grep -h '"metric"' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $f)', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'map', d['phase_ms_avg']['map'], 'agg', d['phase_ms_avg']['agg'], 'hits', d.get('stats',{}).get('lds_hits'), 'ok', d['verified_vs_oracle'])"
done
[ -f gpurun_out/ablate.log ] && grep -v amdgpu.ids gpurun_out/ablate.log | cut -c1-70
