"""K4 on the GPU (csrc/hip/gob.hip): gob value messages for batches of int
structs, bit-identical to the host codec (``_core.gob_encode``, which the golden
bytes of tests/test_gob.py pin) in both directions, with per-message status for
malformed input."""
import pytest
import torch

from ptype_amd.ops import gob as G


def _cols(M, nf, seed):
    g = torch.Generator().manual_seed(seed)
    cols = []
    for f in range(nf):
        small = torch.randint(-200, 200, (M,), generator=g)
        big = torch.randint(-(1 << 62), 1 << 62, (M,), generator=g)
        pick = torch.randint(0, 4, (M,), generator=g)
        c = torch.where(pick == 0, torch.zeros_like(small), torch.where(pick == 1, big, small))
        cols.append(c)
    cols[0][:4] = torch.tensor([0, 127, -64, (1 << 63) - 1])  # 1-byte / 2-byte boundaries, max int
    return cols


def test_host_reference_round_trip():
    cols = _cols(300, 3, 1)
    buf, offs = G.encode_structs(cols, 65)
    back, st = G.decode_structs(buf, offs, 3, 65)
    assert not bool(st.any())
    for a, b in zip(cols, back):
        assert torch.equal(a, b)
    # the 2-field calculator Args{A, B}: zero fields are omitted, as Go does
    b2, o2 = G.encode_structs([torch.tensor([7, 0]), torch.tensor([8, 0])], 65)
    assert bytes(b2.tolist()) == bytes.fromhex("07ff82010e011000" "03ff8200") and o2.tolist() == [0, 8, 12]


@pytest.mark.gpu
@pytest.mark.parametrize("nf,M", [(1, 5000), (2, 200_003), (3, 70_001), (8, 4099)])
def test_gpu_encode_matches_host_codec(nf, M):
    cols = _cols(M, nf, 10 + nf)
    ref_buf, ref_offs = G.encode_structs_ref(cols, 65)
    buf, offs = G.encode_structs([c.cuda() for c in cols], 65)
    assert torch.equal(offs.cpu(), ref_offs)
    assert torch.equal(buf.cpu(), ref_buf)
    back, st = G.decode_structs(buf, offs, nf, 65)
    assert not bool(st.any())
    for a, b in zip(cols, back):
        assert torch.equal(a, b.cpu())


@pytest.mark.gpu
def test_gpu_decode_flags_malformed_messages():
    cols = _cols(64, 2, 3)
    buf, offs = G.encode_structs_ref(cols, 65)
    buf = buf.clone()
    o = offs.tolist()
    buf[o[1] + 2] = 0x84          # message 1: type id 66 (zz 132 = 0x84 after the 0xff count byte)
    buf[o[2]] = buf[o[2]] + 1     # message 2: length byte one too large -> truncated
    # message 3: field delta 16 -> field 15, beyond the 2 fields
    bad = torch.cat([buf[:o[3]], torch.tensor([4, 0xff, 0x82, 0x10, 0x00], dtype=torch.uint8)])
    offs3 = torch.tensor(o[:4] + [o[3] + 5], dtype=torch.int64)
    ref_c, ref_st = G.decode_structs_ref(bad, offs3, 2, 65)
    c, st = G.decode_structs(bad.cuda(), offs3.cuda(), 2, 65)
    assert st.cpu().tolist() == ref_st.tolist()
    assert st.cpu().tolist()[:4] == [G.STATUS_OK, G.STATUS_WRONG_TYPE, G.STATUS_TRUNCATED, G.STATUS_BAD_FIELD]
    for a, b in zip(ref_c, c):
        assert torch.equal(a, b.cpu())
