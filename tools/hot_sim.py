"""hot_sim.py — offline model of k_mark_walk's hot level-1 rows (diagnostic tool, not part of the
product): the share of a C_syn sample's Han occurrences (U+3400..U+9FFF, the runes the fast path
looks up) that a 512-slot table covers, for the library's greedy direct-mapped table
(jb_image.cpp build_hot_rows: runes by summed key frequency, slot = jb_hot_slot) and for other
placements of the same or more rows.  Usage: python tools/hot_sim.py [sample MiB]
"""
import collections
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gen"))
import synth  # noqa: E402

MIB = int(sys.argv[1]) if len(sys.argv) > 1 else 32
s = synth.Synth()
d = tempfile.mkdtemp(prefix="hot_sim_")
dict_path, _ = s.write_files(d)
buf, off, _ = s.corpus(synth.KIND_DOCS, 0, target_bytes=MIB << 20)
text = bytes(buf[:int(off[-1]) if len(off) else len(buf)]).decode("utf-8", errors="replace")
occ = collections.Counter(ch for ch in text if 0x3400 <= ord(ch) <= 0x9FFF)
tot = sum(occ.values())
score = collections.Counter()  # build_hot_rows' score: each key's frequency on every rune of the key
for line in open(dict_path, encoding="utf-8"):
    p = line.split()
    if len(p) >= 2 and int(p[1]) > 0:
        for ch in p[0]:
            score[ch] += int(p[1])


def slot(r):  # jb_hot_slot
    return ((r * 0x9E3779B1) & 0xFFFFFFFF) >> 23


def cov(chs):
    return sum(occ[c] for c in chs) / tot


ranked = [ch for ch, _ in sorted(score.items(), key=lambda kv: (-kv[1], ord(kv[0]))) if 0x3400 <= ord(ch) <= 0x9FFF]
for n in (512, 1024, 2048):
    print(f"ideal top-{n}: {cov(ranked[:n]):.4f}")
tab = {}
for ch in ranked:
    tab.setdefault(slot(ord(ch)), ch)
print(f"direct-mapped 512 (the library): {cov(tab.values()):.4f}; top-512 runes holding a slot:",
      sum(1 for c in ranked[:512] if tab.get(slot(ord(c))) == c))
for ways, shift in ((2, 24), (4, 25)):
    sets = collections.defaultdict(list)
    for ch in ranked:
        st = ((ord(ch) * 0x9E3779B1) & 0xFFFFFFFF) >> shift
        if len(sets[st]) < ways:
            sets[st].append(ch)
    print(f"{ways}-way {512 // ways}x{ways}: {cov([c for v in sets.values() for c in v]):.4f}")
tab2 = {}
for ch in ranked:
    r = ord(ch)
    for sl in (slot(r), ((r * 0x85EBCA6B + 0x9E37) & 0xFFFFFFFF) >> 23):
        if sl not in tab2:
            tab2[sl] = ch
            break
print(f"two hash choices 512: {cov(tab2.values()):.4f}")
print(f"sample {MIB} MiB: {len(occ)} distinct Han runes, {tot} occurrences")
