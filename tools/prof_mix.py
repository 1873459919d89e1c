"""Runs the configs[3] mix (bench.py --workload mix, one GPU) for rocprofv3:
one encode+decode round trip (checked), then ENC encodes and DEC decodes,
each call preceded by a marker dispatch (a 64-sample rpp_pcm_unpack_kernel),
so that tools/pmc_mix_summary.py can attribute every dispatch to its call.
Usage: python tools/prof_mix.py [gib] [enc] [dec] [decode path: auto|fused|segmented]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from dwarfs_amd import codec, parallel  # noqa: E402
from dwarfs_amd.pcm import PcmSampleEndianness as E, PcmSamplePadding as P, PcmSampleSignedness as S  # noqa: E402
from dwarfs_amd.pcm import PcmSampleTransformer  # noqa: E402

gib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
n_enc = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n_dec = int(sys.argv[3]) if len(sys.argv) > 3 else 2
path = sys.argv[4] if len(sys.argv) > 4 else "auto"
dev = torch.device("cuda", 0)
mix = bench.mix_block_mib(gib)
x, offs, ns = bench.make_mix_shard(mix, 0, len(mix), dev)
cfg = codec.CodecConfig(128, 1, "big", 0)
pipe = parallel.ShardPipeline(cfg, x, offs, ns, decode_options=codec.DecodeOptions(path=path))
pipe.step()
torch.cuda.synchronize()
pipe.check(x)
mk = PcmSampleTransformer(E.Little, S.Signed, P.Msb, 2, 16)
mk_src = torch.zeros(128, dtype=torch.uint8, device=dev)
mk_dst = torch.empty(64, dtype=torch.int32, device=dev)


def marker():
    mk.unpack(mk_dst, mk_src)


for _ in range(n_enc):
    marker()
    pipe.encode()
for _ in range(n_dec):
    marker()
    pipe.decode()
marker()
torch.cuda.synchronize()
print(f"prof_mix: {len(mix)} blocks, {int(np.sum(ns)) * 2 / 2**30:.2f} GiB, {n_enc} encodes, {n_dec} decodes, "
      f"decode path {path}")
