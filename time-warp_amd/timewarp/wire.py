"""BinaryP wire sizes (src/Control/TimeWarp/Rpc/Message.hs:155-202) for
bandwidth-aware delay models.

A BinaryP message is `put header >> put (RawData raw)` with
`raw = runPut (put (messageName' r) >> put r)` (Message.hs:166-181); Data.Binary
puts a strict or lazy ByteString as an Int64 length followed by its bytes, a
Text as its UTF-8 ByteString, an Int as 8 bytes, and a Generic product as its
fields in order.  The emulation carries typed payload words, not bytes; these
sizes only turn a message into a transmission time that a scenario adds to the
per-link delays (delay = propagation + bytes / bandwidth).
"""
import math
import struct
from typing import Sequence, Union

INT_BYTES = 8  # Data.Binary Int / Int64


def bytestring_size(n: int) -> int:
    """put (ByteString of n bytes): Int64 length + bytes."""
    return INT_BYTES + int(n)


def text_size(s: str) -> int:
    """put (Text): the UTF-8 ByteString."""
    return bytestring_size(len(s.encode("utf-8")))


def binaryp_size(name: str, content_bytes: int, header_bytes: int = 0) -> int:
    """Bytes on the wire of a BinaryP message named `name` whose Binary content
    encodes to `content_bytes` (Message.hs:166-181; header () = 0 bytes)."""
    raw = text_size(name) + int(content_bytes)
    return int(header_bytes) + bytestring_size(raw)


def bench_message_size(name: str, payload: int) -> int:
    """bench/Network Ping/Pong `MsgId Payload` (Commons.hs:49-70): an Int and a
    lazy ByteString of `payload` bytes."""
    return binaryp_size(name, INT_BYTES + bytestring_size(payload))


def transmission_us(n_bytes: int, bytes_per_s: float) -> int:
    """Serialization time of n_bytes at the link bandwidth, whole µs (ceil)."""
    if bytes_per_s <= 0:
        raise ValueError("bandwidth must be positive")
    return int(math.ceil(n_bytes * 1_000_000 / bytes_per_s))


# ------------------------------------------------------- reference encoder
# A direct Data.Binary-style encoder, used by the tests to pin the sizes above.
Value = Union[int, bytes, str, Sequence]


def encode_binary(v: Value) -> bytes:
    if isinstance(v, bool):
        raise TypeError("no Bool on this wire")
    if isinstance(v, int):
        return struct.pack(">q", v)
    if isinstance(v, bytes):
        return struct.pack(">q", len(v)) + v
    if isinstance(v, str):
        return encode_binary(v.encode("utf-8"))
    return b"".join(encode_binary(x) for x in v)  # Generic product: fields in order


def encode_binaryp(name: str, fields: Sequence) -> bytes:
    raw = encode_binary(name) + encode_binary(list(fields))
    return encode_binary(raw)  # header () puts nothing
