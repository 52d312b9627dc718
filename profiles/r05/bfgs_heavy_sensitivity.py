import sys, time, numpy as np
sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo/mm-admm_amd/python')
import mmadmm_amd as mx, oracle_py
m=mx.MeshData.rect(2,707)
res={}
for pm,cm in [(1,1),(0,0),(1,0),(0,1)]:
    oracle_py.set_pow_mode(pm)
    om=oracle_py.Mesh(2,m.Xp,m.F,m.mask)
    O=oracle_py.Integrator(om,1,0.055,0.5,1.0,nthreads=8,cgMode=cm)
    xs=[]
    for s in range(4):
        O.step(10,-1.0); xs.append(O.get("x").copy())
    res[(pm,cm)]=xs; print(pm,cm,"done",time.strftime("%X"),flush=True)
    np.savez("/tmp/bfgs_heavy_sens_%d%d.npz"%(pm,cm), *xs)
ref=res[(0,0)]
for k,xs in res.items():
    print(k, ["%.3e"%(np.abs(a-b).max()/np.abs(b).max()) for a,b in zip(xs,ref)], flush=True)
