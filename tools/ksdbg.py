import sys, numpy as np
sys.path.insert(0,'.'); sys.path.insert(0,'tests')
from fhe_amd import binfhe as bf
from oracle_lib import Restatement
ps,m=bf.STD128,bf.GINX
P=bf.params(ps,m)
keys=bf.keygen(ps,m,5)
e=bf.GateEngine(ps,m)
rows=P.ksk_rows
for name,A,B in [("ones",np.ones(rows*P.n,np.uint64),np.ones(rows,np.uint64)),
                 ("rowid",(np.arange(rows,dtype=np.uint64)[:,None]*0+np.arange(P.n,dtype=np.uint64)[None,:]).ravel()&16383,np.zeros(rows,np.uint64)),
                 ("rowval",np.repeat(np.arange(rows,dtype=np.uint64)&16383,P.n),np.zeros(rows,np.uint64))]:
    e.load_keys(keys.bsk,A,B)
    a=np.zeros((2,P.N),np.uint64); b=np.array([5,9],np.uint64)
    a[1,:]=np.arange(P.N)%P.qKS
    ga,gb=e.keyswitch(a,b)
    O=Restatement(ps,m)
    oa,ob=O.keyswitch(A,B,a,b)
    print(name,'gpu',ga[:,:6],gb,'\n   ref',oa[:,:6],ob)
