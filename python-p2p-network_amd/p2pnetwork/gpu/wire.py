"""Wire codec bridge: engine broadcasts <-> the packets real p2pnetwork peers exchange.

Restates the framing of ``NodeConnection`` (p2pnetwork/nodeconnection.py) so that payloads
handed to hooks in compat mode are the objects a TCP peer would have received, and so that
engine deliveries can be turned into bytes for real peers:

* ``encode_packet``  -- ``NodeConnection.send`` (nodeconnection.py:107-160): str -> encoded
  text, dict -> ``json.dumps`` text, bytes as is; other types are not sendable (None, the
  reference drops them with a debug message, :158-160); optional compression
  (``compress``, :49-82) = base64(compressed + algorithm tag) + 0x02; every packet ends in
  EOT 0x04.
* ``parse_packet``   -- ``NodeConnection.parse_packet`` (:167-184): a trailing 0x02 means
  compressed (``decompress``, :84-105); then utf-8 text parsed as JSON if it is JSON, else
  the text; undecodable bytes stay bytes.
* ``split_stream``   -- the receive loop's framing (:204-214), including its quirk: the loop
  runs ``while eot_pos > 0``, so an empty packet (EOT at position 0) stops delivery for the
  rest of the buffer.
* ``StreamTap``      -- an engine run as the per-connection byte streams real peers running
  the dedup relay would write, round by round (pinned byte for byte by the wire_* fixtures,
  produced with the reference's own NodeConnection.send).
"""
import base64
import ctypes
from collections import defaultdict
import bz2
import json
import lzma
import zlib

import numpy as np

EOT_CHAR = b"\x04"    # nodeconnection.py:36
COMPR_CHAR = b"\x02"  # nodeconnection.py:39
COMPRESSIONS = ("none", "zlib", "bzip2", "lzma")


def compress(data: bytes, compression: str):
    """base64(compressed + tag) like nodeconnection.py:49-82; None for an unknown algorithm."""
    if compression == "zlib":
        return base64.b64encode(zlib.compress(data, 6) + b"zlib")
    if compression == "bzip2":
        return base64.b64encode(bz2.compress(data) + b"bzip2")
    if compression == "lzma":
        return base64.b64encode(lzma.compress(data) + b"lzma")
    return None


def decompress(packet: bytes) -> bytes:
    """Inverse of ``compress`` (nodeconnection.py:84-105): the tag at the end selects the
    algorithm; a failing or unknown one leaves the base64-decoded bytes as they are."""
    raw = base64.b64decode(packet)
    try:
        if raw[-4:] == b"zlib":
            return zlib.decompress(raw[:-4])
        if raw[-5:] == b"bzip2":
            return bz2.decompress(raw[:-5])
        if raw[-4:] == b"lzma":
            return lzma.decompress(raw[:-4])
    except Exception:
        pass
    return raw


def encode_body(data, encoding_type="utf-8"):
    """The bytes ``send`` puts before the markers, or None if the type is not sendable
    (str / dict / bytes only, nodeconnection.py:113-160; a dict json cannot encode is None)."""
    if isinstance(data, str):
        return data.encode(encoding_type)
    if isinstance(data, dict):
        try:
            return json.dumps(data).encode(encoding_type)
        except TypeError:
            return None
    if isinstance(data, bytes):
        return data
    return None


def encode_packet(data, encoding_type="utf-8", compression="none"):
    """One framed packet exactly as ``NodeConnection.send`` writes it to the socket, or None
    when the reference would send nothing."""
    body = encode_body(data, encoding_type)
    if body is None:
        return None
    if compression == "none":
        return body + EOT_CHAR
    if not body:  # the reference's ratio report divides by len(data) (nodeconnection.py:80);
        return None  # the ZeroDivisionError is caught by send (:122), which stops the link
    c = compress(body, compression)
    if c is None:
        return None
    return c + COMPR_CHAR + EOT_CHAR


def parse_packet(packet: bytes):
    """The object ``node_message`` receives for one packet (without the EOT)."""
    if packet.find(COMPR_CHAR) == len(packet) - 1:
        packet = decompress(packet[:-1])
    try:
        text = packet.decode("utf-8")
    except UnicodeDecodeError:
        return packet
    try:
        return json.loads(text)
    except json.decoder.JSONDecodeError:
        return text


def split_stream(buffer: bytes):
    """(packets, rest): the packets the receive loop delivers from ``buffer`` and the bytes it
    keeps for later -- with the reference's ``eot_pos > 0`` condition (nodeconnection.py:211)."""
    packets = []
    eot = buffer.find(EOT_CHAR)
    while eot > 0:
        packets.append(buffer[:eot])
        buffer = buffer[eot + 1:]
        eot = buffer.find(EOT_CHAR)
    return packets, buffer


def round_trip(data, encoding_type="utf-8", compression="none"):
    """What a peer's ``node_message`` receives when ``data`` is sent over one connection:
    ``(True, obj)``, or ``(False, None)`` when nothing would be sent."""
    pkt = encode_packet(data, encoding_type, compression)
    if pkt is None:
        return False, None
    packets, _ = split_stream(pkt)
    if not packets:  # empty body: the EOT at position 0 delivers nothing (quirk above)
        return False, None
    return True, parse_packet(packets[0])


class StreamTap:
    """The NodeConnection byte streams of an engine run.

    Feed it every round's first receipts in round order (``GraphNetwork.deliveries()`` after
    each step, origination first).  ``feed`` returns the bytes each peer writes on each of its
    connections in that round -- what a real p2pnetwork peer running the dedup relay puts on
    the socket: one ``encode_packet(payload)`` per ``Node.send_to_node`` (node.py:114-120 ->
    NodeConnection.send, nodeconnection.py:107-160), flood to every connection but the sender
    (node.py:106-112), gossip to the k Philox-chosen ones.  Sends lost to churn are counted but
    carry no bytes (nodeconnection.py:123-126).

    Byte order on one connection = the order the sender relays its first receipts, which is
    the order it received them: origins in message order; later, by sender (the parent,
    processed in ascending id) and, within one sender's stream, in that sender's own relay
    order of the round before.  Static topology (no update_edges during the tapped run)."""

    def __init__(self, graph, payloads, mode="flood", fanout=3, gossip_seed=0,
                 churn_threshold=0, churn_seed=0, msg_id_base=0, compression="none"):
        from . import _lib
        self._lib = _lib
        self.graph, self.mode, self.k = graph, mode, int(fanout)
        self.gseed, self.thr, self.cseed = int(gossip_seed), int(churn_threshold), int(churn_seed)
        self.base = int(msg_id_base)
        self.packets = [encode_packet(p, compression=compression) for p in payloads]
        self.round = 0
        self._order = {}  # peer -> {msg: position in its relay order of the previous round}

    def _targets(self, v, m, parent):
        nb = self.graph.neighbours(v)
        if self.mode == "flood":
            return [int(u) for u in nb if u != parent]
        out = np.zeros(max(self.k, 1), dtype=np.uint32)
        n = self._lib.check(self._lib.lib().p2pg_gossip_targets(
            self.round, int(v), self.base + int(m), len(nb), self.k, self.gseed,
            out.ctypes.data_as(ctypes.c_void_p)))
        return [int(nb[j]) for j in out[:n]]

    def _lost(self, a, b):
        return self.thr and self._lib.lib().p2pg_churn_lost(self.round, int(a), int(b), self.thr,
                                                            self.cseed) != 0

    def feed(self, deliveries):
        """(streams, attempted) for the sends of the round whose first receipts these are:
        streams = {(sender, receiver): bytes} (arriving next round), attempted = the
        send_to_node calls made (lost ones included)."""
        peer = np.asarray(deliveries.peer, dtype=np.int64)
        msg = np.asarray(deliveries.msg, dtype=np.int64)
        par = np.asarray(deliveries.parent, dtype=np.int64)
        if self.round == 0:
            key = [(v, m) for v, m in zip(peer, msg)]
        else:
            key = [(v, p, self._order[p][m]) for v, m, p in zip(peer, msg, par)]
        streams = defaultdict(bytearray)
        order = defaultdict(dict)
        attempted = 0
        for i in sorted(range(len(peer)), key=key.__getitem__):
            v, m, p = int(peer[i]), int(msg[i]), int(par[i])
            order[v][m] = len(order[v])
            pkt = self.packets[m]
            for u in self._targets(v, m, p):
                attempted += 1
                if pkt is not None and not self._lost(v, u):
                    streams[(v, u)] += pkt
        self._order = order
        self.round += 1
        return {k: bytes(b) for k, b in streams.items()}, attempted
