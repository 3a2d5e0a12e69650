#!/bin/bash
# M0: capture real MI355X box facts (read-only) into gpurun_out/m0/
set -u
O=gpurun_out/m0
mkdir -p $O
id > $O/id.txt 2>&1
ls -l /dev/kfd /dev/dri > $O/dev.txt 2>&1
ls -l /sys/class/kfd/kfd/topology/nodes/ > $O/kfd_nodes.txt 2>&1
for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "== $n"; cat $n/properties 2>/dev/null | head -60; cat $n/gpu_id 2>/dev/null; done > $O/kfd_props.txt 2>&1
timeout -k 5 60 amd-smi list --json > $O/amdsmi_list.json 2>$O/amdsmi_list.err
timeout -k 5 60 amd-smi static --json > $O/amdsmi_static.json 2>$O/amdsmi_static.err
timeout -k 5 60 amd-smi metric --json > $O/amdsmi_metric.json 2>$O/amdsmi_metric.err
timeout -k 5 60 amd-smi xgmi --json > $O/amdsmi_xgmi.json 2>$O/amdsmi_xgmi.err
timeout -k 5 60 amd-smi topology --json > $O/amdsmi_topo.json 2>$O/amdsmi_topo.err
timeout -k 5 60 amd-smi partition --json > $O/amdsmi_partition.json 2>$O/amdsmi_partition.err
timeout -k 5 60 amd-smi process --json > $O/amdsmi_process.json 2>$O/amdsmi_process.err
timeout -k 5 60 rocm-smi --showtopo --json > $O/rocmsmi_topo.json 2>&1
timeout -k 5 60 rocm-smi --showallinfo --json > $O/rocmsmi_all.json 2>&1
timeout -k 5 60 rocminfo > $O/rocminfo.txt 2>&1
env | grep -E 'ROCR|HIP|HSA|CUDA|GPU' > $O/env.txt
echo "ROCR_VISIBLE_DEVICES=${ROCR_VISIBLE_DEVICES:-unset}" >> $O/env.txt
timeout -k 5 120 python -c "
import time,json
t=time.time()
import amdsmi
amdsmi.amdsmi_init()
hs=amdsmi.amdsmi_get_processor_handles()
out={'n':len(hs),'init_s':time.time()-t,'devs':[]}
for h in hs:
  d={}
  for f in ['amdsmi_get_gpu_device_uuid','amdsmi_get_gpu_device_bdf','amdsmi_get_gpu_asic_info','amdsmi_get_gpu_kfd_info','amdsmi_get_gpu_enumeration_info','amdsmi_get_gpu_compute_partition','amdsmi_get_gpu_memory_partition','amdsmi_get_gpu_total_ecc_count','amdsmi_get_gpu_activity','amdsmi_get_power_info','amdsmi_get_gpu_xgmi_link_status']:
    try: d[f]=getattr(amdsmi,f)(h)
    except Exception as e: d[f]='ERR '+repr(e)
  try: d['mem_total']=amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM)
  except Exception as e: d['mem_total']='ERR '+repr(e)
  for s in ['EDGE','HOTSPOT','VRAM']:
    for m in ['CURRENT','CRITICAL','EMERGENCY']:
      try: d['temp_%s_%s'%(s,m)]=amdsmi.amdsmi_get_temp_metric(h, getattr(amdsmi.AmdSmiTemperatureType,s), getattr(amdsmi.AmdSmiTemperatureMetric,m))
      except Exception as e: d['temp_%s_%s'%(s,m)]='ERR '+repr(e)
  out['devs'].append(d)
print(json.dumps(out, default=str, indent=1))
" > $O/amdsmi_py.json 2>$O/amdsmi_py.err
timeout -k 5 200 python -c "
import time; t=time.time(); import torch; t1=time.time(); n=torch.cuda.device_count(); x=torch.ones(1,device='cuda'); torch.cuda.synchronize(); t2=time.time()
print('import',t1-t,'init',t2-t1,'n',n, torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
" > $O/torch.txt 2>&1
echo done
