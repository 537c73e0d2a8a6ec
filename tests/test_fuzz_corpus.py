"""lneto's own stack fuzz corpus as parity input (VERDICT r5 "Next" 4).

tests/golden/fuzz_frames.json holds the 208 frames of
x/xnet/testdata/fuzz/FuzzStackPacketHTTP (a real TCP/HTTP exchange between
two lneto stacks plus the fuzzer's mutations: truncated, zero-length, VLAN,
ARP and garbage EtherTypes, wrong lengths and sums), made by
tests/golden/make_fuzz_frames.py.  The fuzz harness regenerates a frame's
IPv4 and TCP checksums with fixIPTCPCRCs (x/xnet/xnet_fuzz_test.go:150-185,
restated as oracle.fix_ip_tcp_crcs) before the stack sees it.

On these frames, raw and fixed:
* the receive verdicts (host lnx_ingress_verdict; device
  lnx_ingress_verify_batch and lnx_rx_verify_batch, with and without the FCS)
  equal oracle.ingress_verdict (internet/stack-ethernet.go:139-165,
  internet/stack-ip4.go:100-167) under every flag;
* the transmit checksum step (oracle.tx_checksum, host lnx_tx_checksum,
  device lnx_tx_checksum_batch and lnx_tx_finish_batch) regenerates exactly
  the bytes fixIPTCPCRCs writes, for every frame the harness can fix (its
  total length inside the frame: the step sets total length = len - 14, so
  each frame is taken up to 14 + total length);
* the FCS of every frame (ethernet/crc.go:19-21), including the empty one."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = [0, O.VERIFY_EVIL_BIT, O.VERIFY_ICMP, O.VERIFY_EVIL_BIT | O.VERIFY_ICMP]


def _frames():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "fuzz_frames.json")))
    return [bytes.fromhex(f["hex"]) for f in d["frames"]]


def _fixed():
    return [O.fix_ip_tcp_crcs(f)[0] for f in _frames()]


def _fixable():
    """(raw frame taken to 14 + total length, the fixed frame taken the same) for every frame fixIPTCPCRCs fixes."""
    out = []
    for f in _frames():
        g, ok = O.fix_ip_tcp_crcs(f)
        if ok:
            n = 14 + ((f[16] << 8) | f[17])
            out.append((f[:n], g[:n]))
    return out


def test_corpus_shape():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "fuzz_frames.json")))
    fr = _frames()
    assert len(fr) == 208 and all(isinstance(f["pktnum"], int) for f in d["frames"])
    assert min(map(len, fr)) == 0 and max(map(len, fr)) <= 1518
    kinds = {f[12:14] for f in fr if len(f) >= 14}
    assert {b"\x08\x00", b"\x08\x06", b"\x81\x00"} <= kinds  # IPv4, ARP, VLAN among the mutations
    fixed = [O.fix_ip_tcp_crcs(f)[1] for f in fr]
    assert fixed.count(True) >= 100 and None not in fixed


def test_fixed_frames_pass_the_checksum_stage():
    """After fixIPTCPCRCs the TCP/IPv4 frames no longer fail the IPv4 header or
    TCP sums: none of the fixable frames gets ErrBadCRC (3); raw, most mutated
    frames do."""
    raw = [O.ingress_verdict(f) for f in _frames()]
    assert raw.count(O.ERR_BAD_CRC) > 100
    for f in _frames():
        g, ok = O.fix_ip_tcp_crcs(f)
        if ok:
            assert O.ingress_verdict(g) != O.ERR_BAD_CRC


def test_tx_checksum_regenerates_fix_ip_tcp_crcs():
    """The transmit checksum step (encapsulate4's IPv4 header and TCP sums,
    internet/stack-ip4.go:202-228) writes the bytes fixIPTCPCRCs writes: oracle
    and the library's host path (lnx_tx_checksum)."""
    import ctypes
    import lneto_amd as L
    pairs = _fixable()
    assert len(pairs) >= 100
    for raw, want in pairs:
        got, st = O.tx_checksum(raw)
        assert st == 0 and got == want
        buf = ctypes.create_string_buffer(raw, len(raw))
        assert L.lib.lnx_tx_checksum(buf, len(raw)) == 0 and buf.raw == want


@pytest.mark.parametrize("flags", FLAGS)
def test_host_verdicts_on_the_corpus(flags):
    import lneto_amd as L
    for f in _frames() + _fixed():
        assert L.lib.lnx_ingress_verdict(f, len(f), flags, None) == O.ingress_verdict(f, flags), f.hex()


def _packed(frames, cuda, extra=0):
    import torch
    from lneto_amd import synth
    lens = np.array([len(f) for f in frames], dtype=np.int64)
    off = synth.offsets_from_lengths(lens).astype(np.int64) + 3
    buf = np.zeros(int(off[-1]) + 8 + extra, dtype=np.uint8)
    for f, o in zip(frames, off[:-1]):
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return torch.from_numpy(buf).to(cuda), torch.from_numpy(off).to(cuda), off


@pytest.mark.gpu
@pytest.mark.parametrize("flags", FLAGS)
def test_gpu_ingress_verdicts_on_the_corpus(cuda, flags):
    import lneto_amd as L
    for frames in (_frames(), _fixed()):
        d, o, _ = _packed(frames, cuda)
        got = L.ingress_verify_batch(d, o, flags=flags).cpu().numpy()
        want = np.array([O.ingress_verdict(f, flags) for f in frames], dtype=np.uint8)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:10]]


@pytest.mark.gpu
@pytest.mark.parametrize("flags", FLAGS)
def test_gpu_rx_verify_on_the_corpus(cuda, flags):
    """Each frame with its LE FCS appended (a third of them with one FCS byte
    flipped): fcs_ok and the verdict of the frame without its FCS; and the raw
    frames under LNX_RX_NO_FCS (no CRC, the verdict of the whole frame)."""
    import struct
    import lneto_amd as L
    rng = np.random.default_rng(flags)
    for frames in (_frames(), _fixed()):
        flip = rng.random(len(frames)) < 0.33
        withfcs = []
        for f, fl in zip(frames, flip):
            fcs = bytearray(struct.pack("<I", O.crc32(f)))
            if fl:
                fcs[int(rng.integers(0, 4))] ^= 0x08
            withfcs.append(f + bytes(fcs))
        d, o, _ = _packed(withfcs, cuda)
        ok, verdict = L.rx_verify_batch(d, o, flags=flags)
        assert (ok.cpu().numpy() == (~flip).astype(np.uint8)).all()
        want = np.array([O.ingress_verdict(f, flags) for f in frames], dtype=np.uint8)
        got = verdict.cpu().numpy()
        assert (got == want).all(), np.nonzero(got != want)[0][:10]
        d, o, _ = _packed(frames, cuda)
        ok, verdict = L.rx_verify_batch(d, o, flags=flags | L.RX_NO_FCS)
        assert (ok.cpu().numpy() == 1).all() and (verdict.cpu().numpy() == want).all()


@pytest.mark.gpu
def test_gpu_tx_checksum_regenerates_fix_ip_tcp_crcs(cuda):
    """lnx_tx_checksum_batch and lnx_tx_finish_batch (LNX_TX_CHECKSUM; and with
    LNX_TX_FCS: then padded and FCS appended as oracle.fcs_append) on every
    fixable corpus frame give fixIPTCPCRCs' bytes."""
    import torch
    import lneto_amd as L
    pairs = _fixable()
    cap = 1600
    n = len(pairs)
    for mode in ("tx_checksum", "tx_finish1", "tx_finish3"):
        buf = np.zeros(n * cap + 8, dtype=np.uint8)
        for k, (raw, _) in enumerate(pairs):
            buf[k * cap + 5:k * cap + 5 + len(raw)] = np.frombuffer(raw, np.uint8)
        d = torch.from_numpy(buf).to(cuda)
        starts = torch.from_numpy(np.arange(n, dtype=np.int64) * cap + 5).to(cuda)
        lens = torch.tensor([len(r) for r, _ in pairs], dtype=torch.int32, device=cuda)
        if mode == "tx_checksum":
            st = L.tx_checksum_batch(d, starts, lens)
        else:
            st = L.tx_finish_batch(d, starts, lens, cap - 5, flags=1 if mode == "tx_finish1" else 3)
        st, out, ln = st.cpu().numpy(), d.cpu().numpy(), lens.cpu().numpy()
        for k, (raw, want) in enumerate(pairs):
            if mode == "tx_finish3":
                want, _ = O.fcs_append(want, cap - 5)
            got = out[k * cap + 5:k * cap + 5 + int(ln[k])].tobytes()
            assert int(st[k]) == 0 and got == want, (mode, k)


@pytest.mark.gpu
def test_gpu_fcs_of_the_corpus(cuda):
    """CRC-32 of every corpus frame (the empty one included) through the plain
    and the short-frames entries."""
    import lneto_amd as L
    frames = _frames()
    d, o, _ = _packed(frames, cuda)
    want = np.array([O.crc32(f) for f in frames], dtype=np.uint32)
    for short in (False, True):
        got = L.crc32_batch(d, o, short_frames=short).cpu().numpy().view(np.uint32)
        assert (got == want).all(), np.nonzero(got != want)[0][:10]
