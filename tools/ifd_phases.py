# Per-block phase timestamps of an IFD_DBG build of k_ifd (tools/gpu_r3w.sh):
# phase durations, block lifetime, concurrency. Usage: ifd_phases.py <dir with {zipf,text}_dbg.bin>
import numpy as np, sys
DIR = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r3w"
for w in ("zipf","text"):
    d=np.fromfile(f"{DIR}/{w}_dbg.bin",dtype=np.uint64).reshape(-1,8).astype(np.int64)
    T=d[:,:7].copy(); info=d[:,7]
    t0=T[:,0].min(); T=T-t0  # 10 ns units
    nb=len(T)
    print(w, "blocks",nb, "kernel span us", (T[:,6].max())/100)
    ph=["stage","decode","fix","->agg","lookback","write"]
    for k in range(6):
        a,b=k,k+1
        m = (T[:,a]>=0)&(T[:,b]>0)
        if k==3: pass
        x=(T[m,b]-T[m,a])/100
        print(f"  {ph[k]:8s} mean {x.mean():7.2f} p50 {np.median(x):7.2f} p90 {np.percentile(x,90):7.2f} p99 {np.percentile(x,99):7.2f} max {x.max():8.2f}")
    life=(T[:,6]-T[:,0])/100
    print("  life mean",life.mean(),"p50",np.median(life))
    # start order
    st=T[:,0]; inv=np.sum(np.diff(st)<0); print("  start inversions",inv, "slow lanes total", (info&0xffffffff).sum())
    # concurrency
    ev=np.concatenate([np.stack([T[:,0],np.ones(nb)],1),np.stack([T[:,6],-np.ones(nb)],1)])
    ev=ev[np.argsort(ev[:,0],kind='stable')]; c=np.cumsum(ev[:,1]); print("  max concurrency",c.max(), "mean", c[len(c)//4:3*len(c)//4].mean())
    # per 10% of blocks start time
    for q in (0.1,0.5,0.9): i=int(q*nb); print(f"  block {i} start {T[i,0]/100:.1f} end {T[i,6]/100:.1f}")
