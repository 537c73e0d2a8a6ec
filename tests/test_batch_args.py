"""Argument checks of the Python batch wrappers (lneto_amd/__init__.py `_Batch`):
the C-ABI reads offsets as uint64, lengths/seeds as uint32 and bytes as uint8,
so a tensor of another width would be reinterpreted; tensors on different
devices, or an output that is too small, would touch foreign memory."""
import pytest
import torch

import lneto_amd as L


def test_host_tensors_rejected():
    d = torch.zeros(16, dtype=torch.uint8)
    o = torch.tensor([0, 4, 8], dtype=torch.int64)
    with pytest.raises(L.LnetoError, match="device tensor"):
        L.crc32_batch(d, o)
    with pytest.raises(L.LnetoError, match="device tensor"):
        L.sum16_batch(d, o[:2].contiguous(), torch.tensor([4, 4], dtype=torch.int32))


def test_required_none_rejected():
    """Only the optional arguments (d_min_off, d_seed) may be None."""
    o = torch.tensor([0, 4, 8], dtype=torch.int64)
    with pytest.raises(L.LnetoError, match="d_bytes is required"):
        L.crc32_batch(None, o)
    with pytest.raises(L.LnetoError, match="d_off is required"):
        L.crc32_search_batch(torch.zeros(8, dtype=torch.uint8), None)
    with pytest.raises(L.LnetoError, match="d_len is required"):
        L.sum16_batch(torch.zeros(8, dtype=torch.uint8), o, None)


@pytest.mark.gpu
def test_wrong_widths_rejected(cuda):
    d = torch.zeros(64, dtype=torch.uint8, device=cuda)
    o64 = torch.tensor([0, 4, 8], dtype=torch.int64, device=cuda)
    with pytest.raises(L.LnetoError, match="d_off must be i64"):
        L.crc32_batch(d, o64.to(torch.int32))
    with pytest.raises(L.LnetoError, match="d_bytes must be u8"):
        L.crc32_batch(d.to(torch.int32), o64)
    ln = torch.tensor([4, 4], dtype=torch.int32, device=cuda)
    with pytest.raises(L.LnetoError, match="d_len must be i32"):
        L.sum16_batch(d, o64[:2].contiguous(), ln.to(torch.int64))
    with pytest.raises(L.LnetoError, match="d_seed must be i32"):
        L.sum16_batch(d, o64[:2].contiguous(), ln, ln.to(torch.int64))
    with pytest.raises(L.LnetoError, match="d_min_off must be i64"):
        L.crc32_search_batch(d, o64, ln)
    with pytest.raises(L.LnetoError, match="d_len holds"):
        L.sum16_batch(d, o64[:2].contiguous(), ln[:1].contiguous())
    with pytest.raises(L.LnetoError, match="not.*contiguous|contiguous"):
        L.crc32_batch(d, torch.zeros(6, dtype=torch.int64, device=cuda)[::2])


@pytest.mark.gpu
def test_out_checked(cuda):
    d = torch.zeros(64, dtype=torch.uint8, device=cuda)
    o = torch.tensor([0, 4, 8, 12], dtype=torch.int64, device=cuda)
    with pytest.raises(L.LnetoError, match="out holds 2"):
        L.crc32_batch(d, o, out=torch.empty(2, dtype=torch.int32, device=cuda))
    with pytest.raises(L.LnetoError, match="out must be i32"):
        L.crc32_batch(d, o, out=torch.empty(3, dtype=torch.int64, device=cuda))
    with pytest.raises(L.LnetoError, match="out must be u8"):
        L.fcs_verify_batch(d, o, out=torch.empty(3, dtype=torch.int32, device=cuda))
    out = torch.full((5,), -1, dtype=torch.int32, device=cuda)
    L.crc32_batch(d, o, out=out)
    got = out.cpu().tolist()
    assert got[3:] == [-1, -1] and len(set(got[:3])) == 1  # three CRCs of 4 zero bytes; the rest untouched


@pytest.mark.gpu
def test_explicit_stream(cuda):
    d = torch.arange(256, dtype=torch.uint8, device=cuda)
    o = torch.tensor([0, 100, 256], dtype=torch.int64, device=cuda)
    s = torch.cuda.Stream(device=cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    got = L.crc32_batch(d, o, stream=s)
    s.synchronize()
    import zlib
    b = bytes(range(256))
    assert [x & 0xFFFFFFFF for x in got.cpu().tolist()] == [zlib.crc32(b[:100]), zlib.crc32(b[100:])]
