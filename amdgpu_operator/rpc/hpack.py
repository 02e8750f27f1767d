"""HPACK (RFC 7541) header compression for the operator's HTTP/2 gRPC.

Decoder: every representation a peer may send - indexed fields, literals
with / without / never indexing, dynamic-table size updates - over the static
table and a size-bounded dynamic table, with Huffman-coded strings (Go's
HPACK encoder in the kubelet Huffman-codes a string whenever that is
shorter).  Encoder: literals without indexing, names from the static table
where one matches, raw strings; it never adds to the peer's dynamic table, so
the encoder has no state to keep in step with the peer.

The Huffman code of RFC 7541 Appendix B is canonical: codes are assigned in
order of (length, symbol).  ``_LENGTHS`` holds each symbol's code length and
the codes follow from it; tests/test_rpc.py checks the result against the
RFC's Appendix C examples and the all-ones 30-bit EOS code.
"""

from __future__ import annotations

# RFC 7541 Appendix A
STATIC_TABLE = (
    (":authority", ""), (":method", "GET"), (":method", "POST"), (":path", "/"), (":path", "/index.html"),
    (":scheme", "http"), (":scheme", "https"), (":status", "200"), (":status", "204"), (":status", "206"),
    (":status", "304"), (":status", "400"), (":status", "404"), (":status", "500"), ("accept-charset", ""),
    ("accept-encoding", "gzip, deflate"), ("accept-language", ""), ("accept-ranges", ""), ("accept", ""),
    ("access-control-allow-origin", ""), ("age", ""), ("allow", ""), ("authorization", ""), ("cache-control", ""),
    ("content-disposition", ""), ("content-encoding", ""), ("content-language", ""), ("content-length", ""),
    ("content-location", ""), ("content-range", ""), ("content-type", ""), ("cookie", ""), ("date", ""),
    ("etag", ""), ("expect", ""), ("expires", ""), ("from", ""), ("host", ""), ("if-match", ""),
    ("if-modified-since", ""), ("if-none-match", ""), ("if-range", ""), ("if-unmodified-since", ""),
    ("last-modified", ""), ("link", ""), ("location", ""), ("max-forwards", ""), ("proxy-authenticate", ""),
    ("proxy-authorization", ""), ("range", ""), ("referer", ""), ("refresh", ""), ("retry-after", ""),
    ("server", ""), ("set-cookie", ""), ("strict-transport-security", ""), ("transfer-encoding", ""),
    ("user-agent", ""), ("vary", ""), ("via", ""), ("www-authenticate", ""),
)
_STATIC_NAME_INDEX: dict[str, int] = {}
for _i, (_n, _v) in enumerate(STATIC_TABLE, 1):
    _STATIC_NAME_INDEX.setdefault(_n, _i)
_STATIC_EXACT = {pair: i for i, pair in reversed(list(enumerate(STATIC_TABLE, 1)))}

# Huffman code length of symbols 0..255 and EOS (256), RFC 7541 Appendix B
_LENGTHS = (
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28,  # 0-15
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,  # 16-31
    6, 10, 10, 12, 13, 6, 8, 11, 10, 10, 8, 11, 8, 6, 6, 6,  # ' ' ! " # $ % & ' ( ) * + , - . /
    5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8, 15, 6, 12, 10,  # 0-9 : ; < = > ?
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,  # @ A-O
    7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14, 6,  # P-Z [ \ ] ^ _
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5,  # ` a-o
    6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28,  # p-z { | } ~ DEL
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23,  # 128-143
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,  # 144-159
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23,  # 160-175
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,  # 176-191
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,  # 192-207
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,  # 208-223
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23,  # 224-239
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,  # 240-255
    30,  # EOS
)
EOS = 256


def _canonical_codes(lengths) -> list[int]:
    codes = [0] * len(lengths)
    code, prev = 0, 0
    for length, sym in sorted((n, s) for s, n in enumerate(lengths)):
        code <<= length - prev
        codes[sym] = code
        code += 1
        prev = length
    return codes


CODES = _canonical_codes(_LENGTHS)
# decode map: (length, code) -> symbol
_DECODE = {(n, c): s for s, (n, c) in enumerate(zip(_LENGTHS, CODES))}
_MIN_LEN = min(_LENGTHS)


class HPACKError(ValueError):
    """A header block that cannot be decoded: a COMPRESSION_ERROR for the connection."""


def huffman_encode(data: bytes) -> bytes:
    acc = nbits = 0
    out = bytearray()
    for b in data:
        acc = (acc << _LENGTHS[b]) | CODES[b]
        nbits += _LENGTHS[b]
        while nbits >= 8:
            nbits -= 8
            out.append((acc >> nbits) & 0xFF)
        acc &= (1 << nbits) - 1
    if nbits:  # pad with the EOS prefix (ones)
        out.append(((acc << (8 - nbits)) | ((1 << (8 - nbits)) - 1)) & 0xFF)
    return bytes(out)


def huffman_decode(data: bytes) -> bytes:
    out = bytearray()
    code = length = 0
    for byte in data:
        for shift in range(7, -1, -1):
            code = (code << 1) | ((byte >> shift) & 1)
            length += 1
            if length < _MIN_LEN:
                continue
            sym = _DECODE.get((length, code))
            if sym is None:
                if length > 30:
                    raise HPACKError("invalid Huffman code")
                continue
            if sym == EOS:
                raise HPACKError("EOS in a Huffman-coded string")
            out.append(sym)
            code = length = 0
    # the padding is the most significant bits of EOS (all ones), shorter than a byte
    if length > 7 or code != (1 << length) - 1:
        raise HPACKError("invalid Huffman padding")
    return bytes(out)


def encode_int(out: bytearray, value: int, prefix_bits: int, first: int) -> None:
    """``first``: the bits above the prefix of the first byte."""
    limit = (1 << prefix_bits) - 1
    if value < limit:
        out.append(first | value)
        return
    out.append(first | limit)
    value -= limit
    while value >= 0x80:
        out.append((value & 0x7F) | 0x80)
        value >>= 7
    out.append(value)


def decode_int(buf: bytes, pos: int, prefix_bits: int) -> tuple[int, int]:
    if pos >= len(buf):
        raise HPACKError("truncated integer")
    limit = (1 << prefix_bits) - 1
    value = buf[pos] & limit
    pos += 1
    if value < limit:
        return value, pos
    shift = 0
    while True:
        if pos >= len(buf):
            raise HPACKError("truncated integer")
        b = buf[pos]
        pos += 1
        value += (b & 0x7F) << shift
        if not b & 0x80:
            return value, pos
        shift += 7
        if shift > 28:
            raise HPACKError("integer too large")


def _decode_str(buf: bytes, pos: int) -> tuple[str, int]:
    if pos >= len(buf):
        raise HPACKError("truncated string")
    huff = buf[pos] & 0x80
    n, pos = decode_int(buf, pos, 7)
    if pos + n > len(buf):
        raise HPACKError("truncated string")
    raw = bytes(buf[pos:pos + n])
    if huff:
        raw = huffman_decode(raw)
    return raw.decode("latin-1"), pos + n


class Decoder:
    """One per connection direction: header blocks are decoded in the order they arrive."""

    def __init__(self, max_table_size: int = 4096, max_list_size: int = 256 << 10):
        self.max_allowed = max_table_size  # our SETTINGS_HEADER_TABLE_SIZE
        # decoded size bound (RFC 7541 entry sizes): a small block of indexed
        # references to large table entries must not expand without limit
        self.max_list_size = max_list_size
        self.max_size = max_table_size
        self.table: list[tuple[str, str]] = []  # newest first
        self.size = 0

    def _evict(self) -> None:
        while self.size > self.max_size and self.table:
            n, v = self.table.pop()
            self.size -= len(n) + len(v) + 32

    def _add(self, name: str, value: str) -> None:
        entry = len(name) + len(value) + 32
        if entry > self.max_size:  # an entry larger than the table empties it
            self.table.clear()
            self.size = 0
            return
        self.table.insert(0, (name, value))
        self.size += entry
        self._evict()

    def _get(self, index: int) -> tuple[str, str]:
        if index <= 0:
            raise HPACKError("header index 0")
        if index <= len(STATIC_TABLE):
            return STATIC_TABLE[index - 1]
        i = index - len(STATIC_TABLE) - 1
        if i >= len(self.table):
            raise HPACKError(f"header index {index} out of range")
        return self.table[i]

    def decode(self, block: bytes) -> list[tuple[str, str]]:
        out = []
        pos = 0
        n = len(block)
        total = 0
        while pos < n:
            b = block[pos]
            if b & 0xE0 == 0x20:  # dynamic table size update
                size, pos = decode_int(block, pos, 5)
                if size > self.max_allowed:
                    raise HPACKError(f"table size update {size} above {self.max_allowed}")
                self.max_size = size
                self._evict()
                continue
            if b & 0x80:  # indexed header field
                idx, pos = decode_int(block, pos, 7)
                field = self._get(idx)
            elif b & 0xC0 == 0x40:  # literal with incremental indexing
                idx, pos = decode_int(block, pos, 6)
                name, pos = (self._get(idx)[0], pos) if idx else _decode_str(block, pos)
                value, pos = _decode_str(block, pos)
                self._add(name, value)
                field = (name, value)
            else:  # literal without indexing (0000) / never indexed (0001)
                idx, pos = decode_int(block, pos, 4)
                name, pos = (self._get(idx)[0], pos) if idx else _decode_str(block, pos)
                value, pos = _decode_str(block, pos)
                field = (name, value)
            total += len(field[0]) + len(field[1]) + 32
            if total > self.max_list_size:
                raise HPACKError(f"header list above {self.max_list_size} bytes")
            out.append(field)
        return out


def _put_str(out: bytearray, s: str) -> None:
    raw = s.encode("latin-1")
    encode_int(out, len(raw), 7, 0)
    out += raw


def encode(headers) -> bytes:
    """Literal header fields without indexing (names from the static table
    where one matches); an exact static-table match is sent indexed."""
    out = bytearray()
    for name, value in headers:
        i = _STATIC_EXACT.get((name, value))
        if i is not None:
            encode_int(out, i, 7, 0x80)
            continue
        idx = _STATIC_NAME_INDEX.get(name)
        if idx is not None:
            encode_int(out, idx, 4, 0x00)
        else:
            out.append(0x00)
            _put_str(out, name)
        _put_str(out, value)
    return bytes(out)
