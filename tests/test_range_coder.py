"""Range-coder oracle (c/compress.cs:69-943, restated in oracle/range_coder_oracle.c)
on CPU: the round trip decompress(compress(x)) == x over random, skewed, text-like,
constant and long inputs (long ones wrap the 4096-symbol model, compress.cs:417-441),
plus the 0 returns: empty input, output over the limit.  No GPU."""
import numpy as np
import pytest

import oracle


def corpus(n, seed=1, max_len=3000):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kind = i % 5
        L = int(rng.integers(1, max_len))
        if kind == 0:
            b = rng.integers(0, 256, L, dtype=np.uint8)                     # incompressible
        elif kind == 1:
            b = rng.integers(0, 4, L, dtype=np.uint8)                       # 2 bits of entropy
        elif kind == 2:
            b = np.frombuffer((b"player %d moved to (%d, %d); " % (i, i * 3, i * 7) * 400)[:L], np.uint8)
        elif kind == 3:
            b = np.full(L, i & 0xFF, np.uint8)                              # constant
        else:
            b = (np.cumsum(rng.integers(-2, 3, L)) & 0xFF).astype(np.uint8)  # slowly varying
        out.append(b)
    return out


def pack(msgs):
    lens = np.array([len(m) for m in msgs], np.uint32)
    off = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
    data = np.concatenate(msgs) if msgs else np.zeros(0, np.uint8)
    return data, off, lens


def round_trip(lib, msgs):
    data, off, lens = pack(msgs)
    c, coff, clen = oracle.range_coder_batch(lib, False, data, off, lens, lens * 2 + 64)
    d, doff, dlen = oracle.range_coder_batch(lib, True, c, coff, clen, lens + 16)
    return c, coff, clen, d, doff, dlen


def test_round_trip(oracle_lib):
    msgs = corpus(300)
    c, coff, clen, d, doff, dlen = round_trip(oracle_lib, msgs)
    assert (clen > 0).all()
    for i, m in enumerate(msgs):
        assert int(dlen[i]) == len(m), i
        assert (d[int(doff[i]):int(doff[i]) + len(m)] == m).all(), i
    data, _, lens = pack(msgs)
    # structured inputs shrink, random ones grow a little
    ratio = [int(clen[i]) / len(m) for i, m in enumerate(msgs)]
    assert np.mean(ratio[1::5]) < 0.5 and np.mean(ratio[3::5]) < 0.1


def test_long_inputs_wrap_the_model(oracle_lib):
    msgs = corpus(10, seed=2, max_len=200000)
    msgs = [m for m in msgs if len(m) > 20000] or [np.arange(60000, dtype=np.uint8)]
    c, coff, clen, d, doff, dlen = round_trip(oracle_lib, msgs)
    for i, m in enumerate(msgs):
        assert int(dlen[i]) == len(m) and (d[int(doff[i]):int(doff[i]) + len(m)] == m).all()


def test_zero_returns(oracle_lib):
    msgs = [np.zeros(0, np.uint8), np.arange(256, dtype=np.uint8)]
    data, off, lens = pack(msgs)
    data = np.concatenate([data, np.zeros(16, np.uint8)])
    _, _, clen = oracle.range_coder_batch(oracle_lib, False, data, off, lens, np.array([64, 8], np.uint32))
    assert clen[0] == 0                      # empty input (compress.cs:79-80)
    assert clen[1] == 0                      # output over outLimit (compress.cs:236)
