"""Wire codec bridge (p2pnetwork.gpu.wire) against vectors produced by the reference's own
NodeConnection.send / parse_packet (tests/golden/make_codec_golden.py): exact packet bytes,
framing, and decoded objects, for every payload type and compression the reference has."""
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def untag(d):
    t, v = d["t"], d["v"]
    if t == "bytes":
        return bytes.fromhex(v)
    if t == "tuple":
        return tuple(v)
    if t == "dict_with_tuple":
        return {"tuple": tuple(v["tuple"])}
    return v


def vectors():
    with open(os.path.join(HERE, "golden", "codec_vectors.json")) as f:
        return json.load(f)["vectors"]


@pytest.mark.parametrize("i", range(len(vectors())))
def test_codec_matches_reference(i):
    from p2pnetwork.gpu import wire
    v = vectors()[i]
    data = untag(v["input"])
    pkt = wire.encode_packet(data, compression=v["compression"])
    assert (pkt or b"") == bytes.fromhex(v["packet_hex"])
    packets, rest = wire.split_stream(pkt or b"")
    assert rest == bytes.fromhex(v["rest_hex"])
    got = [wire.parse_packet(p) for p in packets]
    want = [untag(p) for p in v["parsed"]]
    assert got == want
    assert [type(x) for x in got] == [type(x) for x in want]
    ok, obj = wire.round_trip(data, compression=v["compression"])
    assert ok == bool(want)
    if ok:
        assert obj == want[0]


def test_stream_quirk_empty_packet_stops_delivery():
    from p2pnetwork.gpu import wire
    packets, rest = wire.split_stream(b"a\x04\x04b\x04")
    assert packets == [b"a"] and rest == b"\x04b\x04"
