# simulation of k_ntt1024w64<., Sol60> in natural index space: the plan decides folds by the register a
# coefficient occupies in the current layout; compared with the oracle restatement
import sys, numpy as np
sys.path.insert(0, "tests")
from oracle_lib import Restatement
Q=2**60-2**14+1; S=14; M=2**64; N=1024
def mul(y,w,wp):
    assert 0 <= y < M
    yl,yh=y&0xffffffff,y>>32; pl,ph=wp&0xffffffff,wp>>32
    q=yh*ph+((yl*ph)>>32)+((yh*pl)>>32)
    wl,wh=w&0xffffffff,w>>32; p=yl*wl
    rh=((p>>32)+yl*wh+yh*wl-((q&0xffffffff)<<28))&0xffffffff
    r=(((rh<<32)|(p&0xffffffff))+((q<<S)%M)-q)%M
    assert r < 4*Q and r % Q == y*w % Q
    return r
def fold(x): k=x>>60; return (x & (2**60-1)) + (k<<S) - k
def canon(x): f=fold(x); return f-Q if f>=Q else f
kFwdBit=[3,2,1,0,3,2,1,0,1,0]; kInvBit=[0,1,0,1,2,3,0,1,2,3]
def plan64(inv):
    fold_=[[False]*16 for _ in range(10)]; k=[[0]*16 for _ in range(10)]; B=[1]*16
    for st in range(10):
        if (not inv and st in (4,8)) or (inv and st in (2,6)):
            U=max(B); B=[U]*16
        bt=kInvBit[st] if inv else kFwdBit[st]
        for r in range(16):
            if r & (1<<bt): continue
            q=r|(1<<bt)
            if not inv:
                if B[r]+4>16: fold_[st][r]=True; B[r]=2
                B[r]+=4; B[q]=B[r]
            else:
                while B[r]+B[q]>16:
                    e=r if B[r]>=B[q] else q
                    fold_[st][e]=True; B[e]=2
                k[st][r]=B[q]
                B[r]=1 if st==9 else B[r]+B[q]; B[q]=1 if st==9 else 4
    return fold_,k
def reg(x, layout):
    if layout=='A': return x>>6
    if layout=='B': return (x>>2)&15
    return ((x>>8)<<2)|(x&3)
def brev(v,b): return int(format(v,'0%db'%b)[::-1],2)
R=Restatement()
psi=R.L.tfo_root_of_unity(2048,Q)
tab=[pow(psi,brev(i,10),Q) for i in range(N)]
inv_psi=pow(psi,Q-2,Q); tabI=[pow(inv_psi,brev(i,10),Q) for i in range(N)]
ninv=pow(N,Q-2,Q)
def fwd(a):
    F,_=plan64(False); v=list(a)
    for st in range(10):
        bit=9-st; layout='A' if st<4 else 'B' if st<8 else 'C'
        for x in range(N):
            if F[st][reg(x,layout)] and not (x>>bit)&1: v[x]=fold(v[x])
        m=1<<st; t=N>>(st+1)
        for i in range(m):
            w=tab[m+i]; wp=(w<<64)//Q
            for j in range(2*i*t, 2*i*t+t):
                X,Y=v[j],v[j+t]; T=mul(Y,w,wp)
                assert X+4*Q<M
                v[j]=X+T; v[j+t]=X+4*Q-T
    return [canon(x) for x in v]
def inv(a):
    F,K=plan64(True); v=list(a)
    for st in range(10):
        bit=st; layout='C' if st<2 else 'B' if st<6 else 'A'
        for x in range(N):
            if F[st][reg(x,layout)]: v[x]=fold(v[x])
        t=1<<st; m=N>>(st+1)
        for i in range(m):
            w=tabI[m+i]
            if st==9: w=(w*ninv)%Q
            wp=(w<<64)//Q
            for j in range(2*i*t, 2*i*t+t):
                X,Y=v[j],v[j+t]; kk=K[st][reg(j,layout)]
                assert Y < kk*Q and X+Y < M
                d=X+kk*Q-Y
                if st==9:
                    v[j]=canon(mul(X+Y,ninv,(ninv<<64)//Q)); v[j+t]=canon(mul(d,w,wp))
                else:
                    v[j]=X+Y; v[j+t]=mul(d,w,wp)
    return v
rng=np.random.default_rng(1)
xs=[rng.integers(0,Q,N,dtype=np.uint64), np.full(N,Q-1,np.uint64), np.zeros(N,np.uint64)]
for x in xs:
    f=fwd([int(t) for t in x]); ref=R.ntt(Q,psi,x[None,:])[0]
    assert [int(t) for t in ref]==f, "fwd"
    i=inv([int(t) for t in x]); refi=R.ntt(Q,psi,x[None,:],inverse=True)[0]
    assert [int(t) for t in refi]==i, "inv"
print("sim ok", plan64(False)[0][3][:4], plan64(True)[1][9][:8])
