"""Go encoding/gob subset: golden bytes and round trips.

No Go toolchain exists here, so the golden bytes are the ones the gob
specification derives (the Point{22,33} example of encoding/gob's package doc
and the survey's Args/int derivations); parity against a live Go peer is
"unpinned" until a Go capture is available.
"""
from dataclasses import dataclass

from ptype_amd import _core
from ptype_amd.gobtypes import GoSlice, GoStruct, GoUint


@dataclass
class Point:
    X: int
    Y: int


@dataclass
class Args:
    A: int
    B: int


def test_gob_doc_point_example():
    # encoding/gob package documentation: Point{22, 33}
    want = bytes.fromhex(
        "1fff8103010105506f696e7401ff820001020101580104000101590104000000" "07ff82012c014200")
    assert _core.gob_encode([Point(22, 33)]) == want


def test_gob_int_singleton_and_args():
    assert _core.gob_encode([56]).hex() == "03040070"  # reply 56: len 3, int id 2, delta 0, 56<<1
    enc = _core.gob_encode([Args(7, 8)])
    assert enc.endswith(bytes.fromhex("07ff82010e011000"))  # Args{A:7,B:8} value message


def test_gob_request_header_then_args_ids():
    # net/rpc writes Request (type 65) then Args (type 66): Args value uses ff 84
    req = GoStruct("Request", ServiceMethod="Calculator.Multiply", Seq=GoUint(0))
    enc = _core.gob_encode([req, Args(7, 8)])
    assert bytes.fromhex("07ff84010e011000") in enc
    assert b"Request" in enc and b"ServiceMethod" in enc and b"Seq" in enc


def test_gob_zero_fields_omitted_and_roundtrip():
    vals = [Args(0, 5), GoStruct("T", S="", N=-3, F=2.5, B=True, Y=b"\x00\x01", L=[1, -2, 300],
                                 U=GoUint(1 << 40), M={"k": 1}), "hello", 3.25, False, b"raw",
            GoSlice([], proto="")]
    out = _core.gob_decode(_core.gob_encode(vals))
    assert out[0] == GoStruct("Args", A=0, B=5)
    t = out[1]
    assert (t.S, t.N, t.F, t.B, t.Y, t.L, t.U, t.M) == ("", -3, 2.5, True, b"\x00\x01", [1, -2, 300], 1 << 40, {"k": 1})
    assert out[2:6] == ["hello", 3.25, False, b"raw"]
    assert out[6] == []


def test_gob_uint_encoding_boundaries():
    # uint: < 128 one byte, else -(bytecount) then big-endian bytes
    assert _core.gob_encode([GoUint(127)])[-1:] == b"\x7f"
    assert _core.gob_encode([GoUint(256)]).endswith(b"\xfe\x01\x00")
    assert _core.gob_decode(_core.gob_encode([-1, -129, 2**62]))[:3] == [-1, -129, 2**62]
