"""CPU: the prefix_dictionary.gob loader (JB_DICT_GOB, newJiebaPrefixDictionary,
tokenizer.go:439-458) and the serialized image (JB_DICT_IMAGE, jb_save /
jb_image_save).  Host code only: no kernel is launched here.

The real prefix_dictionary.gob is a Git-LFS pointer in the reference
(SURVEY.md Appendix C), so the gob decoder is pinned by tests/gobenc.py (an
independent restatement of the encoding/gob wire format) and by the bytes Go
1.18 writes for a map[string]int type definition; see test_gob_type_definition_bytes.
"""
import os
import random

import pytest

import gobenc
import jiebahip as J
import oracle as O


def _gob_items(dp):
    """The map buildPrefixDictionary makes from dict.txt lines (what the real gob
    holds, tokenizer.go:340-366): words last-wins, proper prefixes with 0."""
    m = {}
    with open(dp, "rb") as f:
        for line in f.read().splitlines():
            w, c = line.split(b" ")[:2]
            m[w] = int(c)
            s = w.decode("utf-8")
            for i in range(1, len(s)):
                m.setdefault(s[:i].encode("utf-8"), 0)
    return m


def test_gob_type_definition_bytes():
    """Go 1.18 `gob.NewEncoder(w).Encode(map[string]int{"a": 1})` starts with this
    type definition (type id 65 = the first user type id)."""
    want = bytes.fromhex("0eff8104 0102ff82 00010c01 040000".replace(" ", ""))
    assert gobenc.type_def_message(65) == want
    assert gobenc.value_message([("a", 1)]) == bytes.fromhex("07ff8200010161 02".replace(" ", ""))


def test_gob_uint_int_encoding():
    assert gobenc.enc_uint(0x7F) == b"\x7f"
    assert gobenc.enc_uint(0x80) == b"\xff\x80"
    assert gobenc.enc_uint(256) == b"\xfe\x01\x00"
    assert gobenc.enc_int(-1) == b"\x01" and gobenc.enc_int(1) == b"\x02"
    assert gobenc.enc_int(-129) == b"\xfe\x01\x01"  # the encoding/gob package doc example
    assert gobenc.enc_int(60_101_967) == gobenc.enc_uint(60_101_967 << 1)


def test_gob_loader_equals_map(syn_small):
    """The gob of buildPrefixDictionary's map loads as exactly that map
    (every entry, freq-0 prefixes included) with size 60,101,967."""
    dp, ep, _ = syn_small
    m = _gob_items(dp)
    items = list(m.items())
    random.Random(3).shuffle(items)  # Go writes maps in random order
    gob = gobenc.encode_map(items)
    assert gobenc.decode_map(gob) == m
    img = J.Image(J.make_config(dict_bytes=gob, emit_path=ep, kind=J.JB_DICT_GOB))
    assert img.dict_info() == (len(m), 60_101_967)
    # the same map as txt lines + the size override: the reference's two loaders agree
    ref = J.Image(J.make_config(dict_bytes=gobenc.map_to_dict_lines(m), emit_path=ep, kind=J.JB_DICT_TXT,
                                size_override=J.JIEBA_SIZE))
    assert ref.dict_info() == (len(m), 60_101_967)
    o = O.Oracle(gobenc.map_to_dict_lines(m).decode(), open(ep, encoding="utf-8").read(), 0, size_override=J.JIEBA_SIZE)
    oitems = o.items()
    rng = random.Random(4)
    for k in rng.sample(sorted(m), 3000):
        s = k.decode("utf-8")
        assert img.lookup(s) == ref.lookup(s), s
        got = img.lookup(s)
        if got is not None:
            assert got[0] == oitems[s]
    # and it equals the dict.txt-with-prefix-semantics image the bench uses
    pre = J.Image(J.make_config(dict_path=dp, emit_path=ep, kind=J.JB_DICT_PREFIX, size_override=J.JIEBA_SIZE))
    assert pre.stats() == img.stats()


def test_gob_size_override_and_other_type_id():
    gob = gobenc.encode_map([("甲", 3), ("甲乙", 0), ("甲乙丙", 200)], type_id=70)
    img = J.Image(J.make_config(dict_bytes=gob, emit_bytes="{}", kind=J.JB_DICT_GOB, size_override=1000))
    assert img.dict_info() == (3, 1000)
    assert img.lookup("甲乙丙")[0] == 200 and img.lookup("甲乙")[0] == 0


def test_gob_negative_and_large_values():
    gob = gobenc.encode_map([("甲", -5), ("乙", 1 << 40), ("丙", 127), ("丁", 128)])
    img = J.Image(J.make_config(dict_bytes=gob, emit_bytes="{}", kind=J.JB_DICT_GOB))
    assert img.dict_info()[0] == 4
    assert img.lookup("乙")[0] == 1 << 40 and img.lookup("丙")[0] == 127 and img.lookup("丁")[0] == 128
    assert img.lookup("甲")[0] == -5


@pytest.mark.parametrize("case", ["empty", "truncated", "not_a_map", "wrong_elem", "value_first", "bad_singleton"])
def test_gob_errors(case):
    good = gobenc.encode_map([("甲", 3)])
    data = {
        "empty": b"",
        "truncated": good[:-2],
        # wireType field 2 (StructT) instead of MapT
        "not_a_map": gobenc._message(gobenc.enc_int(-65) + b"\x03\x00\x00") + gobenc.value_message([("甲", 3)]),
        # map[string]string
        "wrong_elem": gobenc.type_def_message(65, 6, 6) + gobenc.value_message([("甲", 3)]),
        "value_first": gobenc.value_message([("甲", 3)]),
        "bad_singleton": gobenc.type_def_message() + gobenc._message(gobenc.enc_int(65) + b"\x01\x01\x03abc\x06"),
    }[case]
    with pytest.raises(J.JbError) as ei:
        J.Image(J.make_config(dict_bytes=data, emit_bytes="{}", kind=J.JB_DICT_GOB))
    assert ei.value.code == J.JB_EPARSE


def test_gob_trailing_messages_ignored():
    """Decode reads one value; what follows it is not read."""
    gob = gobenc.encode_map([("甲", 3)]) + b"\x05garbage"
    img = J.Image(J.make_config(dict_bytes=gob, emit_bytes="{}", kind=J.JB_DICT_GOB))
    assert img.dict_info() == (1, 60_101_967)


def test_image_roundtrip(syn_small, tmp_path):
    dp, ep, _ = syn_small
    a = J.Image(J.make_config(dict_path=dp, emit_path=ep, kind=J.JB_DICT_PREFIX, size_override=J.JIEBA_SIZE))
    p = str(tmp_path / "syn.jbimg")
    a.save(p)
    b = J.Image(J.make_config(dict_path=p, kind=J.JB_DICT_IMAGE))
    assert b.stats() == a.stats() and b.dict_info() == a.dict_info()
    o = O.Oracle.from_files(dp, ep, 1, size_override=J.JIEBA_SIZE)
    items = o.items()
    for k in random.Random(6).sample(sorted(items), 3000):
        assert a.lookup(k) == b.lookup(k), k
    rng = random.Random(8)
    for _ in range(2000):
        ch = chr(rng.randint(0x3400, 0x9FA5))
        for st in "BMES":
            assert a.emit(st, ch) == b.emit(st, ch)
    # a size override that differs from the saved size rebuilds the weights
    c = J.Image(J.make_config(dict_path=p, kind=J.JB_DICT_IMAGE, size_override=12345))
    k = next(k for k in items if items[k] > 0 and c.lookup(k) is not None)
    assert c.lookup(k)[1] == O.go_log(float(items[k])) - O.go_log(12345.0)


def test_image_corruption_detected(syn_small, tmp_path):
    dp, ep, _ = syn_small
    a = J.Image(J.make_config(dict_path=dp, emit_path=ep))
    p = str(tmp_path / "a.jbimg")
    a.save(p)
    data = bytearray(open(p, "rb").read())
    for mutate in ("flip", "truncate", "magic", "version"):
        d = bytearray(data)
        if mutate == "flip":
            d[len(d) // 2] ^= 0x40
        elif mutate == "truncate":
            d = d[:-7]
        elif mutate == "magic":
            d[0] = ord("X")
        else:
            d[8] = 99
        q = str(tmp_path / f"bad_{mutate}.jbimg")
        with open(q, "wb") as f:
            f.write(d)
        with pytest.raises(J.JbError) as ei:
            J.Image(J.make_config(dict_path=q, kind=J.JB_DICT_IMAGE))
        assert ei.value.code == J.JB_EPARSE, mutate
    assert not os.path.exists(p + ".tmp")


def test_saved_image_reweighed_by_log_table(syn_small, tmp_path, monkeypatch, capfd):
    """A saved image opened with a caller log table (and a new size) is reweighed in
    place (reweigh_image: same trie, new wtab), and its weights equal those of a full
    build from the dictionary with the same table."""
    import math
    dp, ep, _ = syn_small
    a = J.Image(J.make_config(dict_path=dp, emit_path=ep))
    p = str(tmp_path / "syn.jbimg")
    a.save(p)
    keys = [int(x) for x in a.log_keys()]
    size = a.stats()["size"]
    new_size = size + 12345
    rng = random.Random(3)
    # perturb a third of the logarithms by one ulp, either way, and the new size's
    logs = {k: math.nextafter(J.go_log(k), rng.choice([math.inf, -math.inf])) if rng.random() < 0.33 else J.go_log(k)
            for k in keys}
    logs[new_size] = math.nextafter(J.go_log(new_size), math.inf)
    monkeypatch.setenv("JB_DEBUG_BUILD", "1")  # build_image reports its trie placement
    capfd.readouterr()
    re = J.Image(J.make_config(dict_path=p, kind=J.JB_DICT_IMAGE, size_override=new_size, logs=logs))
    assert "trie placement" not in capfd.readouterr().err  # reweighed, not rebuilt
    full = J.Image(J.make_config(dict_path=dp, emit_path=ep, size_override=new_size, logs=logs))
    assert re.stats()["cap"] == a.stats()["cap"]  # the saved trie, not a new placement
    assert _bits(re.stats()["w_absent"]) == _bits(full.stats()["w_absent"])
    o = O.Oracle.from_files(dp, ep, 0)
    items = o.items()
    n = 0
    for k in sorted(items):
        lk = re.lookup(k)
        if lk is None:
            continue
        n += 1
        assert _bits(lk[1]) == _bits(full.lookup(k)[1]), k
        assert _bits(lk[1]) == _bits(logs.get(items[k], J.go_log(items[k])) - logs[new_size]), k
    assert n > 5000


def _bits(x):
    import struct
    return struct.pack("<d", x)


def test_open_image_without_gpu_consumes_image(syn_small):
    """jb_open_image (the Go binding's constructor path) fails loudly without a device
    and takes ownership of the image either way."""
    dp, ep, _ = syn_small
    img = J.Image(J.make_config(dict_path=dp, emit_path=ep))
    logs = {int(k): J.go_log(int(k)) for k in img.log_keys()}
    with pytest.raises(J.JbError) as e:
        J.Tokenizer.from_image(img, logs=logs)
    assert e.value.code == J.JB_EDEVICE
    assert img.h is None  # consumed: no double free at close
    img.close()
