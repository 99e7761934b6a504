import sys, numpy as np
sys.path.insert(0,'tests'); sys.path.insert(0,'oracle'); sys.path.insert(0,'spark-timeseries_amd')
from conftest import load_case
import oracle as O
import sparkts_amd._lib as L
e=L.Engine.get(0)
meta,arr=load_case('c4_515_T512')
s=arr['series']
diffed=np.stack([O.differences_of_order_d(r,1)[1:] for r in s])
init,st=e.hannan_rissanen(diffed,5,5,1)
print("HR ok", st.tolist(), flush=True)
for i in range(len(s)):
    est,ei=O.hannan_rissanen(diffed[i],5,5,1)
    assert est==st[i] and (est!=0 or np.array_equal(ei,init[i])), i
print("HR parity ok", flush=True)
r=e.fit_batch(s,5,1,5,True)
print("fit ok", r['status'].tolist(), flush=True)
