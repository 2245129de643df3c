"""Test infrastructure: encoding/gob for one map[string]int, in Python.

prefix_dictionary.gob (newJiebaPrefixDictionary, /root/reference/tokenizer.go:439-458)
is a Go gob stream of `map[string]int`.  The real file is a Git-LFS pointer here
(SURVEY.md Appendix C), so gob parity is pinned by this independent restatement
of the Go 1.18 encoding/gob wire format (go.mod:3), not by the real bytes:

  message  : uint(byte count) + int(type id) + payload
  id < 0   : wireType of type -id; for a map: field 3 (MapT) = mapType{
             CommonType{Name, Id}, Key, Elem}, each struct ended by delta 0
  id > 0   : a value; a non-struct value starts with the singleton delta 0,
             a map is uint(count) then count x (key, elem)
  uint     : < 0x80 one byte; else byte (256 - n) then n big-endian bytes
  int      : u = v << 1 if v >= 0 else (~v << 1) | 1
  string   : uint(len) + bytes
Predefined ids: int = 2, string = 6; user types start at 65.

`encode_map` writes what `gob.NewEncoder(f).Encode(m)` writes for a map[string]int
(keys in the given order: Go's own order is its random map order, which a
decoder does not see).  `decode_map` reads it back — the oracle side of the
real-data tests uses it to turn a genuine prefix_dictionary.gob into
dictionary lines.
"""


def enc_uint(v):
    if v < 0x80:
        return bytes([v])
    b = v.to_bytes((v.bit_length() + 7) // 8, "big")
    return bytes([256 - len(b)]) + b


def enc_int(v):
    u = (v << 1) if v >= 0 else ((~v) << 1) | 1
    return enc_uint(u)


def _message(payload):
    return enc_uint(len(payload)) + payload


def type_def_message(type_id=65, key_id=6, elem_id=2, name=""):
    """wireType{MapT: &mapType{CommonType{Name, Id}, Key, Elem}} for type `type_id`."""
    common = b""
    field = -1
    if name:
        common += enc_uint(0 - field) + enc_uint(len(name)) + name.encode()
        field = 0
    common += enc_uint(1 - field) + enc_int(type_id) + b"\x00"
    map_t = b"\x01" + common + b"\x01" + enc_int(key_id) + b"\x01" + enc_int(elem_id) + b"\x00"
    wire = b"\x04" + map_t + b"\x00"
    return _message(enc_int(-type_id) + wire)


def value_message(items, type_id=65):
    body = bytearray(enc_int(type_id))
    body += b"\x00"  # singleton field delta
    body += enc_uint(len(items))
    for k, v in items:
        kb = k.encode("utf-8") if isinstance(k, str) else bytes(k)
        body += enc_uint(len(kb)) + kb + enc_int(v)
    return _message(bytes(body))


def encode_map(items, type_id=65):
    """items: iterable of (key, int) pairs."""
    items = list(items)
    return type_def_message(type_id) + value_message(items, type_id)


class _R:
    def __init__(self, b):
        self.b, self.i = b, 0

    def uint(self):
        x = self.b[self.i]
        self.i += 1
        if x < 0x80:
            return x
        n = 256 - x
        v = int.from_bytes(self.b[self.i:self.i + n], "big")
        self.i += n
        return v

    def int(self):
        u = self.uint()
        return ~(u >> 1) if u & 1 else u >> 1


def decode_map(data):
    """The map[string]int of a gob stream, as a dict of bytes -> int."""
    r = _R(data)
    maps = {}
    while True:
        n = r.uint()
        end = r.i + n
        tid = r.int()
        if tid < 0:
            assert r.uint() == 4, "not a map type"
            field, key, elem, common_id = -1, None, None, None
            while True:
                d = r.uint()
                if d == 0:
                    break
                field += d
                if field == 0:
                    f2 = -1
                    while True:
                        d2 = r.uint()
                        if d2 == 0:
                            break
                        f2 += d2
                        if f2 == 0:
                            r.i += r.uint()
                        else:
                            common_id = r.int()
                elif field == 1:
                    key = r.int()
                else:
                    elem = r.int()
            assert r.uint() == 0
            maps[common_id] = (key, elem)
        else:
            assert maps.get(tid) == (6, 2), "not a map[string]int value"
            assert r.uint() == 0
            out = {}
            for _ in range(r.uint()):
                ln = r.uint()
                k = bytes(r.b[r.i:r.i + ln])
                r.i += ln
                out[k] = r.int()
            return out
        r.i = end


def map_to_dict_lines(m):
    """dict.txt lines that NewTokenizer (txt semantics: first wins, no prefixes)
    loads as exactly the map m; pair it with size_override = 60,101,967."""
    return b"".join(k + b" " + str(v).encode() + b"\n" for k, v in m.items())
