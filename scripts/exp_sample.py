import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import cusz_amd as cz
from cusz_amd import datagen
dims=(512,512,512)
x=datagen.smooth3d_torch(dims, seed=2)
r=cz.Resource(cz.F4, dims)
for _ in range(3): r.compress(x.data_ptr(), 1e-4)
r.enable_timing(True)
ts=[]
for _ in range(10):
    r.compress(x.data_ptr(), 1e-4); torch.cuda.synchronize(); ts.append(np.array(r.stage_times()))
t=np.median(np.array(ts),axis=0)*1e3
print(os.environ.get('TAG'), 'predict %.1f book %.1f encode %.1f compress %.1f'%(t[cz.T_PREDICT],t[cz.T_BOOK],t[cz.T_ENCODE],t[cz.T_COMPRESS]))
