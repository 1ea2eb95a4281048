"""Phase stamps (s_memtime per workgroup) of the decode planner's episode kernel and of the
recovery, 1M packets at (10,3,3): dispatch ramp, lifetimes, phase means."""
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
P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
codec = Codec(L, T, B, N)
payload = fill_payload(0, P + T, L, 0x5EED)
er = torch.from_numpy(stream_pattern(P + T, 0)).cuda()
cw, wl = codec.encode(payload)
out, ol = codec.decode(cw, er)
st = torch.zeros(16384 * 8, dtype=torch.int64, device="cuda")
for kernel, name, nph, fn in [(1, "episode", 4, lambda: codec.plan(er)),
                              (4, "recover", 4, lambda: codec.recover(cw, out, ol))]:
    for it in range(3):
        st.zero_()
        lib().fec_debug_stamps(codec._h, kernel, ctypes.c_void_p(st.data_ptr()))
        fn()
        torch.cuda.synchronize()
        lib().fec_debug_stamps(codec._h, kernel, None)
    full = st.cpu().numpy().reshape(-1, 8).astype(np.int64)
    full = full[full[:, 0] > 0]
    s = full[:, :nph]
    if name == "recover":
        cnt = full[:, 4]
        sel = (full[:, 5] > 0) & (full[:, 6] > 0) & (full[:, 7] > 0)
        f = full[sel]
        print(f"   first recovery of wave 0 ({sel.sum()}): loads {np.mean(f[:, 5] - f[:, 7]):.0f} "
              f"(p90 {np.percentile(f[:, 5] - f[:, 7], 90):.0f}), compute+stores {np.mean(f[:, 6] - f[:, 5]):.0f} cycles")
        print(f"   recoveries per wave-0: mean {cnt.mean():.2f} max {cnt.max()}; "
              f"(end - checks) per count: " + str({int(c): round(float(np.mean((s[cnt == c, 3] - s[cnt == c, 2])))) for c in np.unique(cnt)}))
    t0 = s[:, 0].min()
    d = np.diff(s, axis=1)
    life = s[:, -1] - s[:, 0]
    span = s[:, -1].max() - t0
    starts = np.sort(s[:, 0] - t0)
    print(f"{name}: {len(s)} workgroups, span {span} cycles; lifetime mean {life.mean():.0f} "
          f"p50 {np.median(life):.0f} p99 {np.percentile(life, 99):.0f} max {life.max()}", flush=True)
    print("   start offsets p10/p50/p90/max:", [int(np.percentile(starts, q)) for q in (10, 50, 90, 100)],
          " end offsets p50/p90/max:", [int(np.percentile(s[:, -1] - t0, q)) for q in (50, 90, 100)])
    print("   phase means:", [round(float(x)) for x in d.mean(axis=0)],
          " p99:", [round(float(np.percentile(d[:, j], 99))) for j in range(d.shape[1])], flush=True)
