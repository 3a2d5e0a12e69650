#!/bin/bash
# Real-MI355X end-to-end: device library backends, HIP probe via ctypes, bench (config 2), rocprof.
set -u
O=gpurun_out/e2e1
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 120 python -c "
import json
from gpupool.ops import devlib
d = devlib.DeviceLib('amdsmi', node='box')
s = d.snapshot(); print(json.dumps(s, indent=1))
c = devlib.DeviceLib('cli', node='box').snapshot(); print(json.dumps(c, indent=1))
print('amdsmi==cli uuids', [x['uuid'] for x in s['devices']] == [x['uuid'] for x in c['devices']])
" > $O/devlib.json 2>&1 || { echo devlib failed; exit 1; }
timeout -k 10 120 python -c "
import json, time
from gpupool.ops import probe
t=time.time(); n=probe.init(); print('init', n, time.time()-t)
print(probe.hip_uuid_map())
for hbm in (1<<28, 1<<30, 4<<30):
  r = probe.run(0, hbm_bytes=hbm); print(json.dumps(r))
" > $O/probe_ctypes.txt 2>&1 || { echo probe failed; exit 1; }
timeout -k 10 600 python bench.py --gpus 1 --steps 10 --warmup 2 --workdir $PWD/$O/bench1 > $O/bench1.json 2> $O/bench1.err || { echo bench failed; exit 1; }
cat $O/bench1.json
cd /tmp && export TMPDIR=/tmp
export GPUPOOL_AGENT_WRAP="rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o agent --"
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python bench.py --gpus 1 --steps 5 --warmup 1 --workdir $PWD/$O/bench_prof > $O/bench_prof.json 2> $O/bench_prof.err
echo "prof bench rc=$?"
