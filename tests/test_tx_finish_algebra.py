"""The CRC correction of the fused transmit kernel (tx_finish_kernel,
lneto_amd/csrc/rx_verify_kernel.hip) restated on the host and
checked against zlib (the arithmetic of ethernet.CRC32, ethernet/crc.go:19-21,
as StackEthernet.Encapsulate appends it, internet/stack-ethernet.go:200-214).

Phase A folds the frame AS IT IS, padded with zeros to Lp = max(L, 60): its
register R0 = ~CRC32(frame[:Lp]).  The checksum step then changes 16-bit
fields at offsets o_f < 128 by d_f (old XOR new, big-endian on the wire); by
linearity the register of the patched frame is
    R = R0 ^ Z_{Lp - c}( XOR_f Z_{c - o_f}(d_f) ),  c = min(Lp, 128),
with d_f's first byte in the register's low byte and Z_k the register's shift
over k zero bytes, applied by binary powers (the kernel's 16 nibble tables of
Z_{2^m}).  The FCS is ~R, little-endian."""
import random
import zlib

POLY = 0xEDB88320


def _zbit(r: int) -> int:
    return (r >> 1) ^ (POLY if r & 1 else 0)


def _z1(r: int) -> int:  # one zero byte
    for _ in range(8):
        r = _zbit(r)
    return r


def _apply(cols: list[int], x: int) -> int:
    y = 0
    for i in range(32):
        if (x >> i) & 1:
            y ^= cols[i]
    return y


# Z_{2^m}, m < 16, as GF(2) matrices (column i = the image of bit i)
Z2 = [[_z1(1 << i) for i in range(32)]]
for m in range(1, 16):
    Z2.append([_apply(Z2[m - 1], c) for c in Z2[m - 1]])


def zk(k: int, x: int) -> int:
    assert 0 <= k < 1 << 16
    for m in range(16):
        if (k >> m) & 1:
            x = _apply(Z2[m], x)
    return x


def _crc_reg(b: bytes) -> int:  # the register after the frame (init and final XOR undone)
    return ~zlib.crc32(b) & 0xFFFFFFFF


def test_zk_is_the_zero_byte_shift():
    rnd = random.Random(1)
    for _ in range(50):
        x, k = rnd.getrandbits(32), rnd.randrange(0, 3000)
        y = x
        for _ in range(k):
            y = _z1(y)
        assert zk(k, x) == y


def test_field_corrections_match_zlib():
    """Frames of 14..300 bytes and MTU / jumbo-ish lengths, up to four 16-bit
    fields at even and odd offsets below 128 (and inside the frame), random
    old and new values: R0 corrected by the formula is the register of the
    patched frame, so ~R is its FCS."""
    rnd = random.Random(7)
    lengths = list(range(14, 301)) + [1496, 1500, 4000, 9014, 65000]
    for L in lengths:
        frame = bytearray(rnd.getrandbits(8) for _ in range(L))
        Lp = max(L, 60)
        padded = bytes(frame) + bytes(Lp - L)
        R0 = _crc_reg(padded)
        c = min(Lp, 128)
        cand = [o for o in range(0, min(L - 1, 127)) if o + 2 <= min(L, 128)]
        offs = rnd.sample(cand, min(4, len(cand)))
        patched = bytearray(padded)
        D = 0
        for o in offs:
            new = rnd.getrandbits(16)
            old = (patched[o] << 8) | patched[o + 1]
            d = old ^ new
            patched[o], patched[o + 1] = new >> 8, new & 0xFF
            D ^= zk(c - o, ((d >> 8) & 0xFF) | ((d & 0xFF) << 8))  # the field's first byte low
        # (fields are disjoint here; overlapping ones would need their net change)
        if len(set(offs) | {o + 1 for o in offs}) < 2 * len(offs):
            continue
        R = R0 ^ zk(Lp - c, D)
        assert R == _crc_reg(bytes(patched)), (L, offs)
        fcs = (~R & 0xFFFFFFFF).to_bytes(4, "little")
        assert zlib.crc32(bytes(patched) + fcs) == 0x2144DF1C  # the residue of a frame with its FCS
