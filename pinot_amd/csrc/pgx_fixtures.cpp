// libpgx: device memory and copy helpers for callers, and segment-creation helpers (synthetic columns, fixed-bit
// packing, roaring inverted indexes) used by benchmarks and test fixtures -- not on the query path.
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"

extern "C" {

pgx_status pgx_device_alloc(pgx_ctx* ctx, uint64_t bytes, void** out) {
  return guarded([&] {
    if (!ctx || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    void* p = nullptr;
    if (hipMalloc(&p, std::max<uint64_t>(bytes, 256)) != hipSuccess) fail(PGX_ERR_OOM, "hipMalloc failed");
    *out = p;
  });
}

pgx_status pgx_device_free(pgx_ctx* ctx, void* p) {
  return guarded([&] {
    if (!ctx) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (p) hip_check(hipFree(p), "hipFree");
  });
}

pgx_status pgx_copy_to_device(pgx_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  return guarded([&] {
    if (!ctx || !dst || !src) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hip_check(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice), "H2D");
  });
}

pgx_status pgx_copy_to_host(pgx_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
  return guarded([&] {
    if (!ctx || (bytes && (!dst || !src))) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hip_check(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost), "D2H");
  });
}

pgx_status pgx_synth_column_paired(pgx_ctx* ctx, void* device_fwd, int64_t n_rows, int32_t bits, int32_t card,
                                   uint64_t seed, uint64_t pair_seed, uint32_t npairs) {
  return guarded([&] {
    if (!ctx || !device_fwd) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (bits < 1 || bits > 32 || card < 1) fail(PGX_ERR_INVALID_ARG, "bits/card");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    const int64_t n_words = int64_t(padded_fwd_bytes(n_rows, bits) / 4);
    hip_check(pgx_launch_synth(static_cast<uint32_t*>(device_fwd), n_rows, bits, uint32_t(card), seed, n_words, pair_seed, npairs,
                               ctx->stream),
              "synth launch");
    hip_check(hipStreamSynchronize(ctx->stream), "sync");
  });
}

pgx_status pgx_synth_column(pgx_ctx* ctx, void* device_fwd, int64_t n_rows, int32_t bits, int32_t card,
                            uint64_t seed) {
  return pgx_synth_column_paired(ctx, device_fwd, n_rows, bits, card, seed, 0, 0);
}

// ---- segment-creation helpers (benchmark data and fixtures; not on the query path) ----------------------------------

// dictId(row) = splitmix64(seed ^ row * 0x9E3779B97F4A7C15) % card: the same sequence pgx_synth_column packs on device.
pgx_status pgx_synth_dict_ids(uint64_t seed, int64_t n_rows, int32_t card, int32_t* out) {
  return guarded([&] {
    if (!out || n_rows < 0 || card < 1) fail(PGX_ERR_INVALID_ARG, "bad argument");
    for (int64_t r = 0; r < n_rows; ++r) {
      uint64_t x = seed ^ (static_cast<uint64_t>(r) * 0x9E3779B97F4A7C15ull);
      x += 0x9E3779B97F4A7C15ull;
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
      x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
      x ^= x >> 31;
      out[r] = static_cast<int32_t>(x % static_cast<uint64_t>(card));
    }
  });
}

// <col>.bitmap.inv of a column (segment/creator/impl/inv/HeapBitmapInvertedIndexCreator.java:42-81): (card+1) BE int
// offsets, then per dictId the RoaringBitmap 0.5.10 portable serialisation of its doc ids (cookie 12346, no run
// containers; array containers up to 4096 docs, bitmap containers above).  out == NULL (or cap too small) only
// reports the size in *len.
// Segment creation: FixedBitSingleValueWriter's packing (MSB-first, big-endian, no padding between values), 64 bits
// at a time.  out holds ceil(n * bits / 8) bytes.
pgx_status pgx_pack_fixed_bit(const int32_t* ids, int64_t n, int32_t bits, uint8_t* out) {
  return guarded([&] {
    if (bits < 1 || bits > 32 || n < 0 || (n && (!ids || !out))) fail(PGX_ERR_INVALID_ARG, "bad argument");
    const uint64_t nbytes = (uint64_t(n) * uint64_t(bits) + 7) / 8;
    uint64_t acc = 0;  // pending bits, left-aligned count `have`
    int have = 0;
    uint64_t o = 0;
    const uint64_t mask = bits == 32 ? 0xFFFFFFFFull : ((uint64_t(1) << bits) - 1);
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t v = uint64_t(uint32_t(ids[i])) & mask;
      if (have + bits <= 64) {
        acc |= v << (64 - have - bits);
        have += bits;
      } else {
        const int fit = 64 - have;
        acc |= v >> (bits - fit);
        for (int b = 0; b < 8; ++b) out[o++] = uint8_t(acc >> (56 - 8 * b));
        acc = v << (64 - (bits - fit));
        have = bits - fit;
      }
      if (have == 64) {
        for (int b = 0; b < 8; ++b) out[o++] = uint8_t(acc >> (56 - 8 * b));
        acc = 0;
        have = 0;
      }
    }
    for (int b = 0; o < nbytes; ++b) out[o++] = uint8_t(acc >> (56 - 8 * b));
  });
}

pgx_status pgx_inverted_index_build(const int32_t* ids, int64_t n, int32_t card, uint8_t* out, uint64_t cap,
                                    uint64_t* len) {
  return guarded([&] {
    if (!ids || !len || n < 0 || card < 1) fail(PGX_ERR_INVALID_ARG, "bad argument");
    // counting sort of doc ids by dictId
    std::vector<int64_t> start(size_t(card) + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
      if (ids[i] < 0 || ids[i] >= card) fail(PGX_ERR_INVALID_ARG, "dictId out of range");
      ++start[size_t(ids[i]) + 1];
    }
    for (int32_t v = 0; v < card; ++v) start[v + 1] += start[v];
    std::vector<int32_t> docs(static_cast<size_t>(n));
    {
      std::vector<int64_t> pos(start.begin(), start.end() - 1);
      for (int64_t i = 0; i < n; ++i) docs[size_t(pos[ids[i]]++)] = int32_t(i);
    }
    // sizes
    auto bitmap_bytes = [&](int32_t v, std::vector<std::pair<int, int>>* conts) {
      uint64_t b = 8;
      const int64_t a = start[v], e = start[v + 1];
      int64_t i = a;
      while (i < e) {
        const int key = docs[size_t(i)] >> 16;
        int64_t j = i;
        while (j < e && (docs[size_t(j)] >> 16) == key) ++j;
        const int c = int(j - i);
        b += 8 + (c > 4096 ? 8192 : 2 * uint64_t(c));
        if (conts) conts->push_back({key, c});
        i = j;
      }
      return b;
    };
    uint64_t total = 4 * (uint64_t(card) + 1);
    for (int32_t v = 0; v < card; ++v) total += bitmap_bytes(v, nullptr);
    *len = total;
    if (!out || cap < total) return;
    if (total > 0x7FFFFFFFull) fail(PGX_ERR_UNSUPPORTED, "inverted index over 2 GiB");
    auto put32be = [&](uint64_t o, uint32_t x) {
      out[o] = uint8_t(x >> 24); out[o + 1] = uint8_t(x >> 16); out[o + 2] = uint8_t(x >> 8); out[o + 3] = uint8_t(x);
    };
    auto put32le = [&](uint64_t o, uint32_t x) { std::memcpy(out + o, &x, 4); };
    auto put16le = [&](uint64_t o, uint16_t x) { std::memcpy(out + o, &x, 2); };
    uint64_t o = 4 * (uint64_t(card) + 1);
    std::vector<std::pair<int, int>> conts;
    for (int32_t v = 0; v < card; ++v) {
      put32be(4 * uint64_t(v), uint32_t(o));
      conts.clear();
      bitmap_bytes(v, &conts);
      const uint64_t b0 = o;
      const int nc = int(conts.size());
      put32le(o, 12346u);
      put32le(o + 4, uint32_t(nc));
      uint64_t payload = 8 + 8 * uint64_t(nc);
      for (int k = 0; k < nc; ++k) {
        put16le(o + 8 + 4 * k, uint16_t(conts[k].first));
        put16le(o + 8 + 4 * k + 2, uint16_t(conts[k].second - 1));
        put32le(o + 8 + 4 * uint64_t(nc) + 4 * k, uint32_t(payload));
        payload += conts[k].second > 4096 ? 8192 : 2 * uint64_t(conts[k].second);
      }
      uint64_t p = o + 8 + 8 * uint64_t(nc);
      int64_t i = start[v];
      for (int k = 0; k < nc; ++k) {
        const int c = conts[k].second;
        if (c > 4096) {
          std::memset(out + p, 0, 8192);
          for (int t = 0; t < c; ++t) {
            const uint32_t lo = uint32_t(docs[size_t(i + t)]) & 0xFFFFu;
            out[p + (lo >> 3)] |= uint8_t(1u << (lo & 7));
          }
          p += 8192;
        } else {
          for (int t = 0; t < c; ++t) put16le(p + 2 * uint64_t(t), uint16_t(uint32_t(docs[size_t(i + t)]) & 0xFFFFu));
          p += 2 * uint64_t(c);
        }
        i += c;
      }
      o = b0 + (p - b0);
    }
    put32be(4 * uint64_t(card), uint32_t(o));
  });
}

}  // extern "C"
