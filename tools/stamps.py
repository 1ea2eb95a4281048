"""Phase-stamp diagnostics of the specialised encode / copy kernels (s_memtime per workgroup)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import L, stream_pattern  # noqa: E402
from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload, lib  # noqa: E402

torch.cuda.set_device(0)
T, B, N = 10, 3, 3
P = 1_000_000
codec = Codec(L, T, B, N)
payload = fill_payload(0, P + T, L, 0x5EED)
er = torch.from_numpy(stream_pattern(P + T, 0)).cuda()
cw, wl = codec.encode(payload)
out, ol = codec.decode(cw, er)
nwg = (P + T + 7) // 8  # smallest tile the codec picks is 8 packets
st = torch.zeros(nwg * 8, dtype=torch.int64, device="cuda")
for kernel, name, nph in [(0, "encode", 5), (3, "copy", 4)]:
    for it in range(3):
        st.zero_()
        lib().fec_debug_stamps(codec._h, kernel, ctypes.c_void_p(st.data_ptr()))
        if kernel == 0:
            codec.encode(payload, out=cw, out_len=wl)
        else:
            codec.copy(cw, er, out=out, out_len=ol)
        torch.cuda.synchronize()
        lib().fec_debug_stamps(codec._h, kernel, None)
    s = st.cpu().numpy().reshape(-1, 8)[:, :nph].astype(np.int64)
    s = s[(s[:, 0] > 0)]
    d = np.diff(s, axis=1)
    life = s[:, -1] - s[:, 0]
    span = s[:, -1].max() - s[:, 0].min()
    print(f"{name}: {len(s)} workgroups, kernel span {span} cycles; per-workgroup lifetime mean "
          f"{life.mean():.0f} p50 {np.median(life):.0f} p99 {np.percentile(life, 99):.0f}")
    print("   phase means (cycles):", [round(float(x)) for x in d.mean(axis=0)],
          " medians:", [round(float(x)) for x in np.median(d, axis=0)])
    # concurrency: average number of resident workgroups
    print("   mean resident workgroups:", round(float(life.sum() / span), 1))
