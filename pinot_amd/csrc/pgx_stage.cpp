// libpgx: segment staging (Loaders / ColumnIndexContainer): forward indexes, dictionaries and their LDS value images,
// inverted indexes and star trees moved to the device (pgx_segment_stage).
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"

namespace pgxh {

// Re-encode a numeric dictionary into an LDS image (DESIGN.md "LDS value images"): the sum of a column over a scan
// is a per-row dictionary lookup (ImmutableDictionaryReader.readValues), which from HBM/L2 is a random 8-byte gather
// per row.  The image makes it an LDS read.  INT/LONG: u32 (value - min) when the card fits 144 KiB, else 64 block
// bases + u16 offsets (frame of reference; exact, checked per block).  FLOAT/DOUBLE: doubles when they fit.
void build_value_image(pgx_ctx* ctx, StagedColumn& c, SharedDict& sd) {
  const int64_t card = c.card;
  const int64_t kMax = 144 * 1024;
  std::vector<uint32_t> img;
  if (c.data_type == PGX_INT || c.data_type == PGX_LONG) {
    const int64_t vmin = *std::min_element(c.ivals.begin(), c.ivals.end());
    const int64_t vmax = *std::max_element(c.ivals.begin(), c.ivals.end());
    const uint64_t range = uint64_t(vmax) - uint64_t(vmin);
    if (range > 0xFFFFFFFFull) return;
    c.vbase = vmin;
    c.vrange = range;
    if (card * 4 <= kMax) {
      img.resize(card);
      for (int64_t i = 0; i < card; ++i) img[i] = uint32_t(uint64_t(c.ivals[i]) - uint64_t(vmin));
      c.img_kind = IMG_U32;
    } else if (card * 2 + 4 * kImgFor16Blocks <= kMax) {
      int sh = 0;
      while ((card + (int64_t(1) << sh) - 1) >> sh > 32) ++sh;  // <= 32 blocks: base reads are bank-conflict free
      bool ok = false;
      std::vector<uint32_t> base;
      for (int tries = 0; tries < 2 && !ok; ++tries, --sh) {
        if (sh < 0 || ((card + (int64_t(1) << sh) - 1) >> sh) > kImgFor16Blocks) break;
        const int64_t nblk = (card + (int64_t(1) << sh) - 1) >> sh;
        base.assign(kImgFor16Blocks, 0);
        ok = true;
        for (int64_t b = 0; b < nblk && ok; ++b) {
          uint64_t lo = ~0ull, hi = 0;
          for (int64_t i = b << sh; i < std::min(card, (b + 1) << sh); ++i) {
            const uint64_t x = uint64_t(c.ivals[i]) - uint64_t(vmin);
            lo = std::min(lo, x);
            hi = std::max(hi, x);
          }
          if (hi - lo > 0xFFFF) ok = false;
          base[b] = uint32_t(lo);
        }
        if (ok) c.img_sh = sh;
      }
      if (!ok) return;
      img.assign(kImgFor16Blocks + (card + 1) / 2, 0);
      std::copy(base.begin(), base.end(), img.begin());
      uint16_t* off = reinterpret_cast<uint16_t*>(img.data() + kImgFor16Blocks);
      for (int64_t i = 0; i < card; ++i)
        off[i] = uint16_t(uint64_t(c.ivals[i]) - uint64_t(vmin) - base[i >> c.img_sh]);
      c.img_kind = IMG_FOR16;
    } else {
      return;
    }
  } else if (c.data_type == PGX_FLOAT || c.data_type == PGX_DOUBLE) {
    if (card * 8 > kMax) return;
    img.resize(card * 2);
    std::memcpy(img.data(), c.dvals.data(), card * 8);
    c.img_kind = IMG_F64;
  } else {
    return;
  }
  c.img_words = int(img.size());
  img.resize((img.size() + 3) & ~size_t(3), 0);  // whole 16-B chunks for the LDS staging copy
  sd.img = DevBuf(ctx, img.size() * 4);
  hip_check(hipMemcpy(sd.img.p, img.data(), img.size() * 4, hipMemcpyHostToDevice), "image H2D");
}

// The narrow aggregation's packed frame-of-reference image (pgx_narrow.hip IMG 4): per block of 2^sh dictIds a u32 base
// (value - vbase), then every dictId's offset from its block's base in b bits, packed LSB-first into dwords (+ 1 pad
// dword for the two-dword read of the last offset).  The block shift is the one giving the smallest image; built only
// if it fits beside sixteen wavefront tables (kNarrowImg4Words), so the aggregation runs 1024-thread workgroups (four
// wavefronts per SIMD) where the 128 KiB FOR16 image allowed 512.  Exact: b covers every block's span.
bool packed_value_image(pgx_ctx* ctx, SharedDict& sd, const std::vector<int64_t>& ivals) {
  std::lock_guard<std::mutex> g(ctx->dict_mu);
  if (sd.pk_state) return sd.pk_state > 0;
  sd.pk_state = -1;
  const int64_t card = int64_t(ivals.size());
  if (!card || !std::is_sorted(ivals.begin(), ivals.end())) return false;
  int best_sh = -1, best_b = 0;
  int64_t best_words = 0;
  for (int sh = 0; sh <= 16; ++sh) {
    const int64_t nblk = (card + (int64_t(1) << sh) - 1) >> sh;
    uint64_t span = 0;
    for (int64_t b = 0; b < nblk; ++b) {  // sorted: a block's span is its last value minus its first
      const int64_t lo = ivals[size_t(b << sh)], hi = ivals[size_t(std::min(card, (b + 1) << sh) - 1)];
      span = std::max<uint64_t>(span, uint64_t(hi) - uint64_t(lo));
    }
    int bits = 1;
    while (bits < 32 && (uint64_t(1) << bits) <= span) ++bits;
    if (bits > 16) continue;
    const int64_t words = nblk + (card * bits + 31) / 32 + 1;
    if (best_sh < 0 || words < best_words) best_sh = sh, best_b = bits, best_words = words;
  }
  if (best_sh < 0 || best_words > kNarrowImg4Words) return false;
  const int64_t nblk = (card + (int64_t(1) << best_sh) - 1) >> best_sh;
  std::vector<uint32_t> img(size_t(best_words), 0u);
  for (int64_t b = 0; b < nblk; ++b) img[size_t(b)] = uint32_t(uint64_t(ivals[size_t(b << best_sh)]) - uint64_t(sd.vbase));
  for (int64_t i = 0; i < card; ++i) {
    const uint64_t off = uint64_t(ivals[size_t(i)]) - uint64_t(ivals[size_t((i >> best_sh) << best_sh)]);
    const uint64_t pos = uint64_t(i) * uint64_t(best_b);
    const size_t w = size_t(nblk + int64_t(pos >> 5));
    const int o = int(pos & 31);
    img[w] |= uint32_t(off << o);
    if (o + best_b > 32) img[w + 1] |= uint32_t(off >> (32 - o));
  }
  img.resize((img.size() + 3) & ~size_t(3), 0u);  // whole 16-B chunks
  sd.pk_img = DevBuf(ctx, img.size() * 4);
  hip_check(hipMemcpy(sd.pk_img.p, img.data(), img.size() * 4, hipMemcpyHostToDevice), "packed image H2D");
  sd.pk_sh = best_sh | (best_b << 5) | int(nblk << 10);
  sd.pk_words = int(best_words);
  sd.pk_state = 1;
  return true;
}

// StarTreeSerDe.writeTreeOffHeapFormat (core/startree/StarTreeSerDe.java:183-328), native (LE) byte order: u64 magic,
// i32 version, i32 header size, i32 #dims, #dims x {i32 index, i32 len, bytes}, i32 #nodes, #nodes x 7 x i32.
// Other star-tree formats (the Java-serialised ON_HEAP tree) leave st_ok false: queries then scan the raw docs.
void parse_star_tree(pgx_segment& seg) {
  const std::vector<uint8_t>& b = seg.star_tree;
  auto rd32 = [&](size_t o) {
    if (o + 4 > b.size()) fail(PGX_ERR_INVALID_ARG, "segment " + seg.name + ": star tree truncated");
    int32_t x;
    std::memcpy(&x, &b[o], 4);
    return x;
  };
  if (b.size() < 24) return;
  uint64_t magic;
  std::memcpy(&magic, b.data(), 8);
  if (magic != 0xBADDA55B00DAD00Dull) return;
  size_t o = 16;
  const int nd = rd32(o);
  o += 4;
  if (nd < 0 || nd > 4096) fail(PGX_ERR_INVALID_ARG, "segment " + seg.name + ": bad star tree header");
  seg.st_dim_name.assign(nd, "");
  for (int i = 0; i < nd; ++i) {
    const int idx = rd32(o), len = rd32(o + 4);
    if (idx < 0 || idx >= nd || len < 0 || o + 8 + size_t(len) > b.size())
      fail(PGX_ERR_INVALID_ARG, "segment " + seg.name + ": bad star tree dimension map");
    seg.st_dim_name[idx].assign(reinterpret_cast<const char*>(&b[o + 8]), size_t(len));
    o += 8 + size_t(len);
  }
  const int nn = rd32(o);
  o += 4;
  if (nn < 1 || o + size_t(nn) * 28 > b.size()) fail(PGX_ERR_INVALID_ARG, "segment " + seg.name + ": bad star tree");
  seg.st_nodes.resize(nn);
  std::memcpy(seg.st_nodes.data(), &b[o], size_t(nn) * 28);
  for (const auto& x : seg.st_nodes)
    if ((x.cbeg != -1 && (x.cbeg < 1 || x.cend < x.cbeg || x.cend >= nn)) || x.dim >= nd)
      fail(PGX_ERR_INVALID_ARG, "segment " + seg.name + ": star tree node out of range");
  seg.st_ok = true;
}

void stage_dict(pgx_ctx* ctx, pgx_segment* seg, const std::vector<uint8_t>& dict_host, StagedColumn& c);
void stage_forward(pgx_ctx* ctx, pgx_segment* seg, const pgx_column_desc& d, bool device_mem, StagedColumn& c,
                   int64_t n, uint64_t need);

void stage_column(pgx_ctx* ctx, pgx_segment* seg, const pgx_column_desc& d, bool device_mem, StagedColumn& c) {
  c.name = d.name ? d.name : "";
  c.data_type = d.data_type;
  c.card = d.cardinality;
  c.bits = d.bits_per_element;
  c.is_sorted = d.is_sorted != 0;
  c.dict_width = d.dict_width;
  c.pad_char = d.pad_char & 0xFF;
  if (c.card < 1) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": cardinality < 1");
  if (c.bits < 1 || c.bits > 32) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": bitsPerElement out of [1,32]");
  if (c.card > 1 && (c.bits < 32) && (int64_t(c.card) - 1) >> c.bits)
    fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": cardinality does not fit bitsPerElement");
  const int64_t n = seg->total_docs;
  const uint64_t need = padded_fwd_bytes(n, c.bits);

  // ---- dictionary (host copy always; device copy for numeric columns) ----
  std::vector<uint8_t> dict_host;
  if (device_mem) {
    dict_host.resize(d.dict_len);
    if (d.dict_len) hip_check(hipMemcpy(dict_host.data(), d.dict, d.dict_len, hipMemcpyDeviceToHost), "dict D2H");
  } else {
    const uint8_t* p = static_cast<const uint8_t*>(d.dict);
    dict_host.assign(p, p + d.dict_len);
  }
  stage_dict(ctx, seg, dict_host, c);
  stage_forward(ctx, seg, d, device_mem, c, n, need);
}

// The v1 dictionary bytes of column c (c.name / data_type / card / dict_width / pad_char set): host values, the
// context-wide shared device copy and value image (SharedDict).
void stage_dict(pgx_ctx* ctx, pgx_segment* seg, const std::vector<uint8_t>& dict_host, StagedColumn& c) {
  const int width = (c.data_type == PGX_INT || c.data_type == PGX_FLOAT) ? 4
                    : (c.data_type == PGX_STRING)                          ? c.dict_width
                                                                           : 8;
  if (width <= 0 || dict_host.size() < uint64_t(width) * c.card)
    fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": dictionary too short");
  c.dict_hash = fnv1a(dict_host.data(), uint64_t(width) * c.card, fnv1a(&c.data_type, sizeof(int)));
  if (c.data_type == PGX_STRING) {
    c.svals.resize(c.card);
    for (int i = 0; i < c.card; ++i) {
      const char* s = reinterpret_cast<const char*>(dict_host.data()) + size_t(i) * width;
      size_t len = width;
      // StringDictionary.get: truncate at the first padding char (metadata; '\0' default, '%' legacy)
      for (size_t k = 0; k < size_t(width); ++k)
        if (s[k] == char(c.pad_char)) { len = k; break; }
      c.svals[i].assign(s, len);
    }
  } else {
    std::vector<uint64_t> enc(c.card);
    if (c.data_type == PGX_INT || c.data_type == PGX_LONG) {
      c.ivals.resize(c.card);
      for (int i = 0; i < c.card; ++i) {
        int64_t v = (c.data_type == PGX_INT) ? int64_t(int32_t(be32(&dict_host[size_t(i) * 4])))
                                             : int64_t(be64(&dict_host[size_t(i) * 8]));
        c.ivals[i] = v;
        enc[i] = uint64_t(v);
      }
    } else {
      c.dvals.resize(c.card);
      for (int i = 0; i < c.card; ++i) {
        double v;
        if (c.data_type == PGX_FLOAT) {
          uint32_t b = be32(&dict_host[size_t(i) * 4]);
          float f;
          std::memcpy(&f, &b, 4);
          v = double(f);  // (double) widening as FloatDictionary.getDoubleValue
        } else {
          uint64_t b = be64(&dict_host[size_t(i) * 8]);
          std::memcpy(&v, &b, 8);
        }
        c.dvals[i] = v;
        std::memcpy(&enc[i], &v, 8);
      }
    }
    std::lock_guard<std::mutex> g(ctx->dict_mu);
    auto& slot = ctx->dicts[c.dict_hash];
    std::shared_ptr<SharedDict> sd = slot.lock();
    if (sd && (sd->data_type != c.data_type || sd->enc != enc)) sd = nullptr;  // hash collision: a private copy
    if (!sd) {
      sd = std::make_shared<SharedDict>();
      sd->data_type = c.data_type;
      sd->dict = DevBuf(ctx, enc.size() * 8);
      hip_check(hipMemcpy(sd->dict.p, enc.data(), enc.size() * 8, hipMemcpyHostToDevice), "dict H2D");
      build_value_image(ctx, c, *sd);
      sd->img_kind = c.img_kind;
      sd->img_sh = c.img_sh;
      sd->img_words = c.img_words;
      sd->vbase = c.vbase;
      sd->vrange = c.vrange;
      sd->enc = std::move(enc);
      if (!slot.lock()) slot = sd;
      seg->device_bytes += sd->enc.size() * 8 + (sd->img.p ? size_t(sd->img_words) * 4 : 0);
    } else {
      c.img_kind = sd->img_kind;
      c.img_sh = sd->img_sh;
      c.img_words = sd->img_words;
      c.vbase = sd->vbase;
      c.vrange = sd->vrange;
    }
    c.shared = sd;
    c.dict_dev = sd->dict.p;
    c.img_dev = sd->img.p;
  }
}

void stage_forward(pgx_ctx* ctx, pgx_segment* seg, const pgx_column_desc& d, bool device_mem, StagedColumn& c,
                   int64_t n, uint64_t need) {
  if (d.is_multi_value) {
    // FixedBitMultiValueWriter / FixedBitMultiValueReader (io/*/impl/v1/FixedBitMultiValue*.java): numChunks BE int
    // chunk offsets, a totalNumValues-bit MSB-first bitset marking every doc's first value, then the values fixed-bit.
    // docsPerChunk = ceil(2048 / (float)(totalNumValues / numDocs)) with the integer division of the reference.
    c.is_mv = true;
    c.is_sorted = false;
    const int64_t tv = d.total_entries;
    if (tv < n || n < 1) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": totalNumberOfEntries < docs");
    c.total_entries = tv;
    const float avg = float(tv / n);
    const int64_t dpc = int64_t(std::ceil(2048.0f / avg));
    const int64_t nchunks = (n + dpc - 1) / dpc;
    const uint64_t head = uint64_t(nchunks) * 4, bs = uint64_t(tv + 7) / 8, raw = (uint64_t(tv) * c.bits + 7) / 8;
    if (d.fwd_len < head + bs + raw) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": multi-value index short");
    std::vector<uint8_t> f(head + bs + raw);
    if (device_mem) hip_check(hipMemcpy(f.data(), d.fwd, f.size(), hipMemcpyDeviceToHost), "mv fwd D2H");
    else std::memcpy(f.data(), d.fwd, f.size());
    std::vector<int32_t> start;
    start.reserve(size_t(n) + 1);
    for (int64_t i = 0; i < tv; ++i)
      if ((f[head + size_t(i >> 3)] >> (7 - (i & 7))) & 1u) start.push_back(int32_t(i));
    if (int64_t(start.size()) != n || start[0] != 0)
      fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": multi-value doc bitset does not mark one start per doc");
    for (int64_t k = 0; k < nchunks; ++k)
      if (int64_t(be32(&f[size_t(k) * 4])) != start[size_t(k * dpc)])
        fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": multi-value chunk offset mismatch");
    start.push_back(int32_t(tv));
    for (int64_t dd = 0; dd < n; ++dd) c.max_mv = std::max<int>(c.max_mv, start[dd + 1] - start[dd]);
    c.mv_start = DevBuf(ctx, start.size() * 4);
    hip_check(hipMemcpy(c.mv_start.p, start.data(), start.size() * 4, hipMemcpyHostToDevice), "mv starts H2D");
    const uint64_t vneed = padded_fwd_bytes(tv, c.bits);
    c.fwd_owned = DevBuf(ctx, vneed);
    hip_check(hipMemset(c.fwd_owned.p, 0, vneed), "memset");
    hip_check(hipMemcpy(c.fwd_owned.p, f.data() + head + bs, raw, hipMemcpyHostToDevice), "mv values H2D");
    c.fwd = c.fwd_owned.as<const uint32_t>();
    seg->device_bytes += vneed + start.size() * 4;
  } else if (c.is_sorted) {
    // Sorted SV column: card x (start,end) BE int pairs (SortedForwardIndexReader / SortedInvertedIndexReader).
    std::vector<uint8_t> pairs(d.sorted_len);
    if (d.sorted_len < uint64_t(c.card) * 8) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": sorted index short");
    if (device_mem) hip_check(hipMemcpy(pairs.data(), d.sorted_pairs, d.sorted_len, hipMemcpyDeviceToHost), "D2H");
    else std::memcpy(pairs.data(), d.sorted_pairs, d.sorted_len);
    c.sorted_first.resize(c.card);
    c.sorted_last.resize(c.card);
    for (int i = 0; i < c.card; ++i) {
      c.sorted_first[i] = int32_t(be32(&pairs[size_t(i) * 8]));
      c.sorted_last[i] = int32_t(be32(&pairs[size_t(i) * 8 + 4]));
    }
    // Materialise a packed fixed-bit view on device so group-by / value reads use the same unpack path.
    std::vector<uint8_t> packed(need, 0);
    for (int id = 0; id < c.card; ++id) {
      for (int64_t r = std::max<int32_t>(0, c.sorted_first[id]); r <= c.sorted_last[id] && r < n; ++r) {
        const int64_t bit0 = r * c.bits;
        for (int k = 0; k < c.bits; ++k) {
          if ((uint32_t(id) >> (c.bits - 1 - k)) & 1u) {
            const int64_t bit = bit0 + k;
            packed[bit >> 3] |= uint8_t(0x80u >> (bit & 7));
          }
        }
      }
    }
    c.fwd_owned = DevBuf(ctx, need);
    hip_check(hipMemcpy(c.fwd_owned.p, packed.data(), need, hipMemcpyHostToDevice), "fwd H2D");
    c.fwd = c.fwd_owned.as<const uint32_t>();
    seg->device_bytes += need;
  } else {
    const uint64_t file_bytes = (uint64_t(n) * c.bits + 7) / 8;
    if (d.fwd_len < file_bytes) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": forward index short");
    if (device_mem && d.fwd_len >= need && (reinterpret_cast<uintptr_t>(d.fwd) & 15) == 0) {
      c.fwd = static_cast<const uint32_t*>(d.fwd);  // referenced in place (caller keeps it alive)
    } else {
      c.fwd_owned = DevBuf(ctx, need);
      hip_check(hipMemset(c.fwd_owned.p, 0, need), "memset");
      hip_check(hipMemcpy(c.fwd_owned.p, d.fwd, file_bytes, device_mem ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice),
                "fwd copy");
      c.fwd = c.fwd_owned.as<const uint32_t>();
      seg->device_bytes += need;
    }
  }
  if (d.inv && d.inv_len) {
    // <col>.bitmap.inv: (card+1) BE int offsets, then concatenated portable roaring bitmaps
    // (segment/creator/impl/inv/HeapBitmapInvertedIndexCreator.java:74-81, BitmapInvertedIndexReader.java:91-117)
    const uint8_t* p = static_cast<const uint8_t*>(d.inv);
    c.inv.assign(p, p + d.inv_len);
    c.has_inverted = true;
    if (d.inv_len < uint64_t(c.card + 1) * 4) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": inverted index short");
    c.inv_off.resize(c.card + 1);
    bool device_ok = true;
    for (int i = 0; i <= c.card; ++i) {
      c.inv_off[i] = be32(p + 4 * size_t(i));
      if (c.inv_off[i] > d.inv_len || (i && c.inv_off[i] < c.inv_off[i - 1]))
        fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": inverted index offsets out of order");
      // The device expansion reads RoaringBitmap 0.5.10's portable no-run format (cookie 12346), all the reference
      // writes (no runOptimize); anything else keeps this column on the dictId-bitset scan path.
      if (i < c.card) {
        const uint32_t o = c.inv_off[i];
        if ((o & 1u) || uint64_t(o) + 8 > d.inv_len) device_ok = false;
        else if ((uint32_t(p[o]) | uint32_t(p[o + 1]) << 8 | uint32_t(p[o + 2]) << 16 | uint32_t(p[o + 3]) << 24) != 12346u)
          device_ok = false;
      }
    }
    if (device_ok) {
      c.inv_dev = DevBuf(ctx, d.inv_len + 16);
      hip_check(hipMemcpy(c.inv_dev.p, p, d.inv_len, hipMemcpyHostToDevice), "inverted index H2D");
      seg->device_bytes += d.inv_len;
    }
  }
  if (c.is_sorted) c.has_inverted = true;  // ColumnDataSourceImpl: sorted columns report an inverted index
}

}  // namespace pgxh
