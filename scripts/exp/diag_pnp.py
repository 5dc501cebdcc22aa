import sys; sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import numpy as np, _oracle as O
from minicv_amd import native as N, synthetic as S
L=N.lib(); O.load()
print("devices", L.mcvDeviceCount())
for n in (4, 300, 5000):
    img,W,inl,K,d,R,t=S.pnp_problem(n,seed=1,outlier_frac=0.3,sigma=0.5)
    pts8=O.pack_pnp(img,W); c8=O.cam8(K,d)
    poses=[(R,t),(R,t+0.01)]
    P=np.ascontiguousarray(np.concatenate([np.concatenate([a.ravel(),b]) for a,b in poses]),np.float64)
    for mode in (0,1):
        c=np.zeros(2,np.int32)
        r=L.mcvTestPnpSweep(pts8.ctypes.data,n,c8.ctypes.data,P.ctypes.data,2,4.0,0,mode,c.ctypes.data)
        print(n,mode,r,c, [O.pnp_count(pts8,c8,a,b,4.0)[0] for a,b in poses])
    try: print("err", L.mcvGetLastError())
    except Exception as e: print(e)
