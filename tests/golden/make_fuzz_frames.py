#!/usr/bin/env python3
"""Writes tests/golden/fuzz_frames.json from lneto's stack fuzz corpus.

Source: /root/reference/x/xnet/testdata/fuzz/FuzzStackPacketHTTP/* — 208 files
in Go's `go test fuzz v1` format, each `int(pktnum)` and `[]byte("...")`: the
Ethernet frames of a real TCP/HTTP exchange between two lneto stacks and the
fuzzer's mutations of them (x/xnet/xnet_fuzz_test.go:19-80 records the seeds
with f.Add(pktnum, frame)).  The output is data only: per corpus file its name,
pktnum and the frame's bytes as hex.  The byte literal is a Go interpreted
string literal as strconv.Quote writes it (printable ASCII as itself, the
escapes \\a \\b \\f \\n \\r \\t \\v \\\\ \\" and \\xNN, octal \\NNN)."""
import json
import os
import re
import sys

SRC = "/root/reference/x/xnet/testdata/fuzz/FuzzStackPacketHTTP"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fuzz_frames.json")
ESC = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92, '"': 34, "'": 39}


def go_bytes(lit: str) -> bytes:
    out, i = bytearray(), 0
    while i < len(lit):
        c = lit[i]
        if c != "\\":
            out += c.encode("utf-8")
            i += 1
            continue
        e = lit[i + 1]
        if e in ESC:
            out.append(ESC[e])
            i += 2
        elif e == "x":
            out.append(int(lit[i + 2:i + 4], 16))
            i += 4
        elif e in "01234567":
            out.append(int(lit[i + 1:i + 4], 8))
            i += 4
        else:
            raise ValueError(f"escape \\{e}")
    return bytes(out)


def parse(text: str) -> tuple[int, bytes]:
    lines = text.splitlines()
    assert lines[0] == "go test fuzz v1", lines[0]
    pkt = int(re.fullmatch(r"int\((-?\d+)\)", lines[1]).group(1))
    lit = re.fullmatch(r'\[\]byte\("(.*)"\)', lines[2]).group(1)
    return pkt, go_bytes(lit)


def main() -> None:
    frames = []
    for name in sorted(os.listdir(SRC)):
        pkt, b = parse(open(os.path.join(SRC, name), encoding="utf-8").read())
        frames.append({"name": name, "pktnum": pkt, "hex": b.hex()})
    json.dump({"source": "lneto x/xnet/testdata/fuzz/FuzzStackPacketHTTP (go test fuzz v1)",
               "generator": "tests/golden/make_fuzz_frames.py", "frames": frames}, open(OUT, "w"), indent=0)
    print(f"{len(frames)} frames -> {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
