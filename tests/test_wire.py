"""Wire codec bridge (p2pnetwork.gpu.wire) against vectors produced by the reference's own
NodeConnection.send / parse_packet (tests/golden/make_codec_golden.py): exact packet bytes,
framing, and decoded objects, for every payload type and compression the reference has."""
import json
import os

import pytest

from conftest import deliveries_from_planes, fixture_streams, load_golden, wire_cases

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


@pytest.mark.parametrize("name", wire_cases())
def test_stream_tap_matches_reference_bytes(name):
    """StreamTap, fed each round's first receipts (here from the fixture's own hop / parent
    planes), reproduces byte for byte what the reference's NodeConnection.send wrote on every
    connection in every round of the harness run -- order of packets on a connection
    included -- and the attempted sends equal the per-round sum of message_count_send."""
    from p2pnetwork.gpu import PeerGraph
    from p2pnetwork.gpu.wire import StreamTap, parse_packet, split_stream
    z = load_golden(name)
    hop, parent = z["hop"], z["parent"]
    M = hop.shape[1]
    tap = StreamTap(PeerGraph(z["rowptr"], z["colidx"]), [{"mid": m} for m in range(M)],
                    mode=str(z["mode"]), fanout=int(z["fanout"]), gossip_seed=int(z["gossip_seed"]),
                    churn_threshold=int(z["churn_threshold"]), churn_seed=int(z["churn_seed"]))
    want = fixture_streams(z)
    for r in range(int(hop.max()) + 1):
        got, attempted = tap.feed(deliveries_from_planes(hop, parent, r))
        assert got == want.get(r, {}), r
        assert attempted == int(z["round_relays"][r])
        # every stream parses back into the payloads, as the receive loop frames them
        for (a, b), buf in got.items():
            pkts, rest = split_stream(buf)
            assert rest == b"" and all(parse_packet(p)["mid"] < M for p in pkts)
