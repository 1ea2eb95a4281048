import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import os, time, ctypes, numpy as np, torch
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload
from fec_erasure_code_unit_test_relay_amd.relay import StateDependentRelay
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern
from fec_erasure_code_unit_test_relay_amd._lib import lib
print('affinity', len(os.sched_getaffinity(0)), 'cpus', os.cpu_count())
torch.cuda.set_device(0)
P=360000
c=Codec(300,10,3,3); cw,_=c.encode(fill_payload(0,P,300,0x5EED))
e1=load_pattern("bin_erasure")[:P].astype(np.uint8); e2=load_pattern("bin_erasure2")[:P].astype(np.uint8)
r=StateDependentRelay(300,10,3,10,3)
ids=np.zeros(P,np.int32); n=ctypes.c_int64(); rb=ctypes.c_int()
def tm(f, k=3):
    f(); torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(k): f()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/k*1e3
print('relay plan', tm(lambda: lib().fec_sdswdf_relay_plan(r._h, e1.ctypes.data_as(ctypes.c_void_p), P, ids.ctypes.data_as(ctypes.c_void_p), None, 0, ctypes.byref(n), ctypes.byref(rb))))
pid, rec = r.relay_plan(e1); hd=np.ascontiguousarray(rec[pid,:11]); fl=np.zeros(P,np.uint8)
print('dest plan', tm(lambda: lib().fec_sdswdf_dest_plan(r._h, e2.ctypes.data_as(ctypes.c_void_p), hd.ctypes.data_as(ctypes.c_void_p), P, ids.ctypes.data_as(ctypes.c_void_p), fl.ctypes.data_as(ctypes.c_void_p), None, 0, ctypes.byref(n), ctypes.byref(rb))))
print('relay batch', tm(lambda: r.relay(cw, e1)))
fr=r.relay(cw,e1)
print('dest batch', tm(lambda: r.destination(fr, e2)))
print('chain', tm(lambda: r.chain(cw, e1, e2)))
