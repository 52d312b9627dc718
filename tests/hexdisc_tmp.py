import numpy as np
def hexdisc(N, R=1.0, cx=0.0, cy=0.0):
    pts=[(cx,cy)]
    for k in range(1,N+1):
        j=np.arange(6*k); th=np.pi/3*(j/k); r=R*k/N
        pts += list(zip(cx+r*np.cos(th), cy+r*np.sin(th)))
    P=np.array(pts)
    def gid(k,s,t):
        if k==0: return 0
        s=(s+t//k)%6; t=t%k
        return 1+3*k*(k-1)+s*k+t
    F=[]
    for k in range(1,N+1):
        for s in range(6):
            for t in range(k):
                F.append((gid(k,s,t),gid(k,s,t+1),gid(k-1,s,t) if k>1 else 0))
            for t in range(k-1):
                F.append((gid(k-1,s,t),gid(k,s,t+1),gid(k-1,s,t+1)))
    F=np.array(F,dtype=np.int32)
    mask=np.full(len(P),2,dtype=np.int32); mask[1+3*N*(N-1):]=1
    return P,F,mask
