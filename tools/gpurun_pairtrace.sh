# one traced NFLX run with the pair kernel; per wave-kind step times and critical-path makeup
mkdir -p gpurun_out
G=${G:-128}
MFHIP_FAST_KERNEL=pair MFHIP_WAVE_TRACE=gpurun_out/wt.txt timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --fast-waves -$G > gpurun_out/b.log 2>&1 || { echo FAIL; tail -3 gpurun_out/b.log; exit 1; }
python - <<PY
import json, numpy as np
d=json.loads(open("gpurun_out/b.log").read().strip().splitlines()[-1])
print("G $G", round(d["value"]/1e6), d["ms_per_step"], d["config"]["pad_records"], d["rmse"])
a=np.loadtxt("gpurun_out/wt.txt",dtype=np.int64); dur=(a[:,7]-a[:,6])*10.0; ns=dur/np.maximum(a[:,4],1)
for kind in (1,2):
    m=a[:,5]==kind
    if m.sum(): print(" kind",kind,"waves",m.sum(),"ns/step",round(float(np.median(ns[m])),1),"mean steps",round(float(a[m,4].mean()),1),"max",a[m,4].max())
sub=a[:,1]*1000+a[:,2]; tot=0; ck=[]
for k in np.unique(sub):
    w=a[sub==k]; tot+=(w[:,7].max()-w[:,6].min())*10; i=np.argmax(w[:,7]); ck.append((w[i,5],w[i,4],(w[i,7]-w[i,6])*10/w[i,4]))
ck=np.array(ck)
print(" sum span ms", tot/1e6, "critical kinds", np.bincount(ck[:,0].astype(int)), "crit steps", ck[:,1].mean(), "crit ns/step", np.median(ck[:,2]))
PY
