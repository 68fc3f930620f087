"""CPU: the C oracle's chain batch (NET_BUF chains walked routine by routine, net_util.c:1545-1687)
agrees with the stream-view restatement on scattered, odd-offset, empty-piece, NULL-chain,
u32-wrapping and self-verifying chains; the binding's bounds checks refuse short buffers."""
import random

import numpy as np
import pytest

import netcsum
import oracle
from chains import make_chain_batch


@pytest.mark.parametrize("pseudo_len", [0, 12, 13, 40])
@pytest.mark.parametrize("op", [0, 1])
def test_oracle_chain_batch_matches_stream_view(pseudo_len, op):
    rng = random.Random(pseudo_len * 2 + op)
    cb = make_chain_batch(rng, 600, pseudo_len=pseudo_len, self_verify=0.5 if op else 0.0)
    got = oracle.batch_chains(cb.base, cb.piece_off, cb.piece_len, cb.chain_first, cb.pseudo, cb.pseudo_stride,
                              cb.pseudo_len, cb.n, op)
    assert np.array_equal(got, cb.expect(op))
    if op:
        assert 0 < int(got.sum()) < cb.n      # both verdicts occur


def test_oracle_chain_batch_u32_wrap():
    rng = random.Random(7)
    cb = make_chain_batch(rng, 24, wrap_chains=12, pseudo_len=13)
    got = oracle.batch_chains(cb.base, cb.piece_off, cb.piece_len, cb.chain_first, cb.pseudo, cb.pseudo_stride,
                              cb.pseudo_len, cb.n, 0)
    assert np.array_equal(got, cb.expect(0))
    # the wrap is real: an unwrapped (mod 65535) sum disagrees for some of these chains
    import oracle_np as onp
    diff = 0
    for i in range(12):
        s = cb.stream(i)
        exact = onp.be_word_sum(s)
        assert exact >= 1 << 32
        diff += onp.fold(exact) != onp.fold(exact & 0xFFFFFFFF)
    assert diff > 0


def test_binding_refuses_short_chain_buffers():
    n = 4
    first = np.zeros(n, np.uint32)                            # needs n + 1 entries
    out = np.zeros(n, np.uint16)
    with pytest.raises(ValueError):
        netcsum.batch_chains(np.zeros(16, np.uint8), np.zeros(1, np.uint64), np.zeros(1, np.uint16), first, None,
                             0, 0, n, out)
    with pytest.raises(ValueError):
        netcsum.batch_chains(np.zeros(16, np.uint8), np.zeros(1, np.uint64), np.zeros(1, np.uint16),
                             np.zeros(n + 1, np.uint32), None, 0, 0, n, np.zeros(n - 1, np.uint16))
