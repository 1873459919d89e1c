import sys, json, ctypes as C
import numpy as np, torch
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from dwarfs_amd import _native as N
from dwarfs_amd import flac as FL
from test_flac import sines
dev = torch.device("cuda:0")
for channels, nbytes, bits in ((2, 2, 16), (8, 4, 24)):
    n = (16 << 20) // (channels * nbytes)
    rng = np.random.default_rng(1)
    x = (sines(channels, n, bits).astype(np.int64) + rng.integers(-8, 9, n * channels))
    x = np.clip(x, -(1 << (bits - 1)), (1 << (bits - 1)) - 1).astype(np.int32)
    xt = torch.from_numpy(x).to(dev)
    L = N.lib()
    frames = (n + 4095) // 4096
    out = torch.empty(frames * int(L.rpp_flac_frame_bound(channels, bits)) + 64, dtype=torch.uint8, device=dev)
    wsb = int(L.rpp_flac_encode_workspace_bytes(n, channels, bits))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    L.rpp_flac_encode(C.c_void_p(xt.data_ptr()), n, channels, bits, C.c_void_p(out.data_ptr()), C.c_void_p(tot.data_ptr()), C.c_void_p(ws.data_ptr()), wsb, C.c_void_p(s.cuda_stream))
    nb = int(tot.item()); body = out[:nb].clone()
    y = torch.empty(n * channels, dtype=torch.int32, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev); nc = torch.zeros(1, dtype=torch.int32, device=dev)
    mc = n // 4096 + nb // 4096 + 64
    wdb = int(L.rpp_flac_decode_workspace_bytes(nb, channels, bits, 4096, mc))
    wd = torch.zeros(wdb, dtype=torch.uint8, device=dev)
    L.rpp_flac_decode(C.c_void_p(body.data_ptr()), nb, channels, bits, 4096, n, C.c_void_p(y.data_ptr()), C.c_void_p(st.data_ptr()), mc, C.c_void_p(wd.data_ptr()), wdb, C.c_void_p(nc.data_ptr()), C.c_void_p(s.cuda_stream))
    torch.cuda.synchronize()
    w = wd.cpu().numpy()
    r16 = lambda b: (b + 15) & ~15
    o = r16(4 * (nb + 1)); pos = w[o:o + 8 * mc].view(np.uint64); o += r16(8 * mc)
    info = w[o:o + 4 * mc].view(np.uint32); o += r16(4 * mc)
    ln = w[o:o + 8 * mc].view(np.uint64); o += r16(8 * mc)
    ok = w[o:o + 4 * mc].view(np.uint32); o += r16(4 * mc)
    redo = w[o:o + 4 * mc].view(np.uint32)
    k = int(nc.item())
    rr = np.nonzero(redo[:k])[0]
    print(json.dumps({"channels": channels, "ncand": k, "frames": frames, "status": int(st.item()), "equal": bool(torch.equal(y, xt)), "redo": len(rr),
                      "redo_pos": [int(pos[i]) for i in rr[:10]], "redo_len": [int(ln[i]) for i in rr[:10]], "redo_bs": [int(info[i]) for i in rr[:10]]}))
    bb = body.cpu().numpy()
    for i in rr[:3]:
        p0 = int(pos[i]); print(bytes(bb[p0:p0+24]).hex())
