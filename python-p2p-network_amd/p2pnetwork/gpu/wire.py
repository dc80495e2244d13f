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
"""
import base64
import bz2
import json
import lzma
import zlib

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
