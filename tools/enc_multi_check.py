"""Diagnostic: segmented encode of batches of k long streams (16 MiB each by
default) against the oracle, k = 1, 2, 4, 8; prints the first differing byte
of every stream that differs.  Usage: python tools/enc_multi_check.py [mib]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import datagen  # noqa: E402
from dwarfs_amd import codec  # noqa: E402
from oracle import oracle as O  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = mib << 19
cfg = codec.CodecConfig(128, 1, "big", 0)
oc = O.cfg(128, 1, True, 0)
rng = np.random.default_rng(5)
blocks = [datagen.poisson_data(rng, n) for _ in range(8)]
wants = [O.encode(oc, b) for b in blocks]
for k in (1, 2, 4, 8, 3, 5):
    for rep in range(3):
        flat = np.concatenate(blocks[:k])
        d = torch.from_numpy(flat.view(np.int16)).to("cuda:0")
        enc = codec.encode_batch(cfg, d, [i * n for i in range(k)], [n] * k)
        torch.cuda.synchronize()
        st = enc.status.cpu().numpy()
        sizes = enc.sizes.cpu().numpy()
        data = enc.data.cpu().numpy()
        bad = []
        for i in range(k):
            got = data[enc.offsets[i]:enc.offsets[i] + sizes[i]].tobytes()
            if got != wants[i]:
                m = min(len(got), len(wants[i]))
                g = np.frombuffer(got[:m], np.uint8)
                w = np.frombuffer(wants[i][:m], np.uint8)
                diff = int(np.argmax(g != w)) if (g != w).any() else m
                bad.append((i, int(st[i]), len(got), len(wants[i]), diff))
        print(f"k={k} rep={rep}: {'OK' if not bad else bad}", flush=True)
