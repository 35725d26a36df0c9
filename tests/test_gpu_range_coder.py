"""GPU parity of the batched range coder (enet_hip_range_compress_device /
_decompress_device, c/compress.cs:69-943) against the oracle: compressed bytes and
sizes bit-exact, decompressed bytes equal to the input, including incompressible,
over-limit, empty and model-wrapping inputs."""
import numpy as np
import pytest

import oracle
from test_gpu_parity import ctx, dctx, dev  # noqa: F401  (fixtures)
from test_range_coder import corpus, pack

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def gpu_coder(ctx, decompress, data, off, lens, limit):  # noqa: F811
    out_off = np.concatenate([[0], np.cumsum(limit.astype(np.uint64))[:-1]]).astype(np.uint64)
    d_out = torch.zeros(int(limit.astype(np.uint64).sum()) + 16, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(len(off), dtype=torch.int32, device="cuda")
    ctx.range_coder_device(decompress, dev(np.concatenate([data, np.zeros(16, np.uint8)])), dev(off), dev(lens),
                           len(off), d_out, dev(out_off), dev(limit), d_len,
                           stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), out_off, d_len.cpu().numpy().view(np.uint32)


def test_compress_matches_oracle(ctx, oracle_lib):  # noqa: F811
    msgs = corpus(2000, seed=7) + [np.zeros(0, np.uint8), np.arange(256, dtype=np.uint8)]
    data, off, lens = pack(msgs)
    limit = lens * 2 + 64
    limit[-1] = 8                                            # over the limit -> 0
    ref, roff, rlen = oracle.range_coder_batch(oracle_lib, False, data, off, lens, limit)
    got, goff, glen = gpu_coder(ctx, False, data, off, lens, limit)
    assert (glen == rlen).all()
    for i in range(len(msgs)):
        a, b = int(roff[i]), int(goff[i])
        assert (got[b:b + int(glen[i])] == ref[a:a + int(rlen[i])]).all(), i
    # GPU decompress of the GPU stream returns the input
    keep = rlen > 0
    cdata = np.concatenate([got[int(goff[i]):int(goff[i]) + int(glen[i])] for i in range(len(msgs)) if keep[i]])
    clens = glen[keep]
    coff = np.concatenate([[0], np.cumsum(clens.astype(np.uint64))[:-1]]).astype(np.uint64)
    dout, doff, dlen = gpu_coder(ctx, True, cdata, coff, clens, lens[keep] + 16)
    for j, i in enumerate(np.nonzero(keep)[0]):
        m = msgs[i]
        assert int(dlen[j]) == len(m) and (dout[int(doff[j]):int(doff[j]) + len(m)] == m).all(), i


def test_decompress_matches_oracle_long(ctx, oracle_lib):  # noqa: F811
    msgs = [m for m in corpus(20, seed=8, max_len=120000)]
    data, off, lens = pack(msgs)
    c, coff, clen = oracle.range_coder_batch(oracle_lib, False, data, off, lens, lens * 2 + 64)
    cdata = np.concatenate([c[int(coff[i]):int(coff[i]) + int(clen[i])] for i in range(len(msgs))])
    coff2 = np.concatenate([[0], np.cumsum(clen.astype(np.uint64))[:-1]]).astype(np.uint64)
    ref, roff, rlen = oracle.range_coder_batch(oracle_lib, True, cdata, coff2, clen, lens + 16)
    got, goff, glen = gpu_coder(ctx, True, cdata, coff2, clen, lens + 16)
    assert (glen == rlen).all() and (rlen == lens).all()
    for i in range(len(msgs)):
        assert (got[int(goff[i]):int(goff[i]) + int(glen[i])] == msgs[i]).all(), i


@pytest.mark.parametrize("lanes,waves,interleave", [(64, 4, 0), (16, 16, 0), (3, 2, 0), (1, 1, 0), (16, 16, 1),
                                                   (5, 3, 1)])
def test_compress_lanes_per_wave(dctx, oracle_lib, monkeypatch, lanes, waves, interleave):  # noqa: F811
    """Any number of active lanes per wave and waves per CU (diagnostics knobs
    ENET_HIP_RC_LANES / _WAVES; 16 x 16 is the product's): the same bytes as the
    oracle, including DGRAMs taken on a lane's later grid-stride turns (3 x 2 and
    1 x 1 launch fewer lanes than the 3000 DGRAMs)."""
    monkeypatch.setenv("ENET_HIP_RC_LANES", str(lanes))
    monkeypatch.setenv("ENET_HIP_RC_WAVES", str(waves))
    monkeypatch.setenv("ENET_HIP_RC_INTERLEAVE", str(interleave))   # (1: symbol-major models)
    msgs = corpus(3000, seed=9) + [np.zeros(0, np.uint8)]
    data, off, lens = pack(msgs)
    limit = lens * 2 + 64
    ref, roff, rlen = oracle.range_coder_batch(oracle_lib, False, data, off, lens, limit)
    got, goff, glen = gpu_coder(dctx, False, data, off, lens, limit)
    assert (glen == rlen).all()
    for i in range(len(msgs)):
        a, b = int(roff[i]), int(goff[i])
        assert (got[b:b + int(glen[i])] == ref[a:a + int(rlen[i])]).all(), i
