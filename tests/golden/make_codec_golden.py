"""Generate tests/golden/codec_vectors.json by driving the REFERENCE's NodeConnection codec.

Runs only in the build container (needs /root/reference, read-only; nothing from it is
copied).  For each (payload, compression) the reference ``NodeConnection.send``
(nodeconnection.py:107-160) writes into an in-memory fake socket; the bytes are split with
the receive loop's framing rule (:204-214) and decoded by the reference
``NodeConnection.parse_packet`` (:167-184).  The fixture records inputs, exact packet bytes
and the decoded objects (type-tagged JSON) -- data only.

Usage:  python tests/golden/make_codec_golden.py
"""
import importlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def tag(x):
    if isinstance(x, bytes):
        return {"t": "bytes", "v": x.hex()}
    if isinstance(x, str):
        return {"t": "str", "v": x}
    return {"t": type(x).__name__, "v": x}  # dict / list / int / float / bool / None


INPUTS = [
    "hello", "", "5", "3.25", '{"a": 1}', "[1, 2]", "null", "true", '"quoted"', "héllo wörld",
    "x" * 5000,
    {"mid": 7, "hop": 2}, {}, {"nested": {"k": [1, 2.5, None, True]}, "s": "t"},
    {"tuple": (1, 2)}, {"big": "y" * 3000},
    b"raw bytes", b"", b"5", b'{"a": 2}', b"\xff\xfe\x00\x01", bytes(range(1, 256)),
    5, 2.5, [1, 2], None, (3, 4),
]
COMPRESSIONS = ["none", "zlib", "bzip2", "lzma", "snappy"]


class _Sock:
    def __init__(self):
        self.out = b""

    def settimeout(self, t):
        pass

    def sendall(self, b):
        self.out += b


class _Main:
    def debug_print(self, m):
        pass


def main():
    sys.path.insert(0, REF)
    nc = importlib.import_module("p2pnetwork.nodeconnection")
    assert os.path.abspath(nc.__file__).startswith(REF), nc.__file__
    vectors = []
    for data in INPUTS:
        for comp in COMPRESSIONS:
            sock = _Sock()
            conn = nc.NodeConnection(_Main(), sock, "peer", "127.0.0.1", 1)
            conn.send(data, compression=comp)
            pkt = sock.out
            # the receive loop's framing (nodeconnection.py:204-214)
            packets, buf = [], pkt
            eot = buf.find(conn.EOT_CHAR)
            while eot > 0:
                packets.append(buf[:eot])
                buf = buf[eot + 1:]
                eot = buf.find(conn.EOT_CHAR)
            parsed = [tag(conn.parse_packet(p)) for p in packets]
            inp = tag(data) if not isinstance(data, tuple) else {"t": "tuple", "v": list(data)}
            if isinstance(data, dict) and "tuple" in data:
                inp = {"t": "dict_with_tuple", "v": {"tuple": list(data["tuple"])}}
            vectors.append({"input": inp, "compression": comp, "packet_hex": pkt.hex(),
                            "parsed": parsed, "rest_hex": buf.hex()})
    with open(os.path.join(HERE, "codec_vectors.json"), "w") as f:
        json.dump({"source": "reference NodeConnection.send / parse_packet", "vectors": vectors}, f,
                  indent=0)
    print(len(vectors), "vectors")


if __name__ == "__main__":
    main()
