// Test harness main (tests/test_unpack.py): random spans with escapes, packed as
// k_span_pack packs them, decoded by unpack_spans into misaligned outputs, checked.

int main() {
  std::mt19937 r(7);
  for (int trial = 0; trial < 40; trial++) {
    uint32_t nt = (trial < 10) ? (r() % 20000) : (r() % 3000000);
    // reference spans: random gaps/lengths with escapes
    std::vector<uint32_t> ts(nt), te(nt);
    uint32_t p = 0;
    double pesc = (trial % 3 == 0) ? 0.3 : (trial % 3 == 1 ? 0.001 : 0.0);
    for (uint32_t i = 0; i < nt; i++) {
      uint32_t g = (r() % 1000) < pesc * 1000 ? 63 + r() % 200 : r() % 63;
      uint32_t l = (r() % 1000) < pesc * 1000 ? 1000 + r() % 100 : 1 + r() % 40;
      ts[i] = p + g; te[i] = ts[i] + l; p = te[i];
    }
    std::vector<uint16_t> pk(nt + 8); std::vector<uint32_t> hdr(nt / kPackBlock + 2); std::vector<uint4> side;
    for (uint32_t i = 0; i < nt; i++) {
      uint32_t pe = i ? te[i - 1] : 0, g = ts[i] - pe, l = te[i] - ts[i];
      if (g >= kPackGapEsc || l >= kPackLenEsc) { pk[i] = 0xFFFF; side.push_back({i, ts[i], te[i], 0}); }
      else pk[i] = (uint16_t)(g | (l << kPackGapBits));
      if ((i & (kPackBlock - 1)) == 0) hdr[i / kPackBlock] = pe;
    }
    std::shuffle(side.begin(), side.end(), r);
    uint64_t base = 1000000007ull * (trial + 1);
    int off = trial % 8;  // misalign the outputs
    std::vector<uint64_t> os(nt + 16), oe(nt + 16 + (trial % 2));
    uint64_t* O = os.data() + off; uint64_t* E = oe.data() + (trial % 2 ? off : off + 1);
    unpack_spans(pk.data(), hdr.data(), side.data(), (uint32_t)side.size(), nt, base, O, E);
    for (uint32_t i = 0; i < nt; i++)
      if (O[i] != base + ts[i] || E[i] != base + te[i]) { printf("trial %d mismatch at %u\n", trial, i); return 1; }
  }
  printf("ok\n"); return 0;
}
