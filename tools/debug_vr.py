import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
torch.cuda.set_device(0)
from fec_erasure_code_unit_test_relay_amd import fill_payload
x = fill_payload(0, 1000, 300)
torch.cuda.synchronize()
print("fill before plan ok", flush=True)
from conftest import load_pattern
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan
v = VrPlan(load_pattern("bin_erasure"), 360000)
print("plan ok", v.lost, flush=True)
x = fill_payload(0, 1000, 300)
torch.cuda.synchronize()
print("fill after plan ok", flush=True)
x = fill_payload(0, v.sent, 300)
torch.cuda.synchronize()
print("fill big ok", flush=True)
