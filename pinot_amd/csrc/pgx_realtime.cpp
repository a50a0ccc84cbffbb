// libpgx: realtime (consuming) segments held on the device and grown in place (include/pgx.h pgx_mutable_*).
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"

extern "C" {

// -------------------------------------------------------------------------------------------------
// Realtime (consuming) segments in place (RealtimeSegmentImpl.java:185-334): per column the docs' arrival-order
// dictIds live in HBM and grow by appends (only the new rows cross PCIe); a snapshot re-packs them on the device through
// the arrival -> sorted dictId map of the column's current dictionary (RealtimeSegmentConverter's shape: sorted
// dictionary, unsorted fixed-bit forward index), so a query costs no host pass over the rows.
// -------------------------------------------------------------------------------------------------
struct pgx_mutable {
  pgx_ctx* ctx = nullptr;
  std::string name;
  int32_t capacity = 0;
  int32_t num_docs = 0;
  struct Col {
    std::string name;
    int data_type = 0;
    bool mv = false, inverted = false;
    DevBuf ids;                  // arrival-order dictIds: one per doc (SV) or per value (MV)
    int64_t ids_cap = 0, nvals = 0;
    DevBuf starts;               // MV: doc d's values are [starts[d], starts[d + 1]) (capacity + 1)
    int max_mv = 0;
    int32_t max_id = -1;         // largest arrival id appended
    int card = 0, dict_width = 0, pad_char = 0;
    std::vector<uint8_t> dict;   // sorted v1 dictionary bytes
    DevBuf remap;                // arrival id -> sorted id
  };
  std::vector<Col> cols;
  mutable std::mutex mu;
};

pgx_status pgx_mutable_create(pgx_ctx* ctx, const char* name, int32_t capacity, int32_t num_columns,
                              const pgx_mutable_column* columns, pgx_mutable** out) {
  return guarded([&] {
    if (!ctx || !columns || !out || capacity < 1 || num_columns < 1) fail(PGX_ERR_INVALID_ARG, "bad argument");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    auto m = std::make_unique<pgx_mutable>();
    m->ctx = ctx;
    m->name = name ? name : "";
    m->capacity = capacity;
    m->cols.resize(num_columns);
    for (int i = 0; i < num_columns; ++i) {
      const pgx_mutable_column& d = columns[i];
      pgx_mutable::Col& c = m->cols[i];
      c.name = d.name ? d.name : "";
      c.data_type = d.data_type;
      c.mv = d.is_multi_value != 0;
      c.inverted = d.has_inverted != 0;
      if (c.mv && c.data_type == PGX_STRING) fail(PGX_ERR_UNSUPPORTED, "multi-value STRING column " + c.name);
      c.ids_cap = c.mv ? std::max<int64_t>(1024, int64_t(capacity)) : capacity;
      c.ids = DevBuf(ctx, size_t(c.ids_cap) * 4);
      if (c.mv) {
        c.starts = DevBuf(ctx, (size_t(capacity) + 1) * 4);
        hip_check(hipMemset(c.starts.p, 0, 4), "memset");
      }
    }
    ctx->refs.fetch_add(1);  // released by pgx_mutable_release
    *out = m.release();
  });
}

pgx_status pgx_mutable_append(pgx_mutable* m, int32_t ndocs, const int32_t* const* ids, const int32_t* const* counts) {
  return guarded([&] {
    if (!m || !ids || ndocs < 0) fail(PGX_ERR_INVALID_ARG, "bad argument");
    std::lock_guard<std::mutex> g(m->mu);
    if (int64_t(m->num_docs) + ndocs > m->capacity) fail(PGX_ERR_INVALID_ARG, "realtime segment " + m->name + " full");
    if (!ndocs) return;
    // Validate every column before any device or host state changes: a rejected batch leaves nvals, starts, max_id
    // and num_docs exactly as they were (no half-appended multi-value column).
    const size_t ncols = m->cols.size();
    std::vector<int64_t> nv(ncols, ndocs);
    std::vector<int32_t> top(ncols, -1), mvmax(ncols, 0);
    for (size_t i = 0; i < ncols; ++i) {
      const pgx_mutable::Col& c = m->cols[i];
      if (!ids[i] || (c.mv && (!counts || !counts[i]))) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": no ids");
      if (c.mv) {
        int64_t at = c.nvals;
        for (int32_t d = 0; d < ndocs; ++d) {
          if (counts[i][d] < 1) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": a multi-value doc needs a value");
          at += counts[i][d];
          mvmax[i] = std::max(mvmax[i], counts[i][d]);
        }
        if (at > 0x7FFFFFFF) fail(PGX_ERR_UNSUPPORTED, "column " + c.name + ": too many values");
        nv[i] = at - c.nvals;
      }
      for (int64_t k = 0; k < nv[i]; ++k) {
        if (ids[i][k] < 0) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": negative dictId");
        top[i] = std::max(top[i], ids[i][k]);
      }
    }
    hip_check(hipSetDevice(m->ctx->device), "hipSetDevice");
    hipStream_t st = m->ctx->stream;
    for (size_t i = 0; i < ncols; ++i) {
      pgx_mutable::Col& c = m->cols[i];
      if (c.mv) {  // the new docs' starts, then the values
        std::vector<int32_t> st_new(ndocs);
        int64_t at = c.nvals;
        for (int32_t d = 0; d < ndocs; ++d) {
          at += counts[i][d];
          st_new[d] = int32_t(at);
        }
        hip_check(hipMemcpyAsync(c.starts.as<int32_t>() + m->num_docs + 1, st_new.data(), size_t(ndocs) * 4,
                                 hipMemcpyHostToDevice, st), "starts H2D");
        hip_check(hipStreamSynchronize(st), "sync");  // st_new is a stack buffer
        if (c.nvals + nv[i] > c.ids_cap) {  // grow the value buffer (doubling)
          int64_t cap = c.ids_cap;
          while (cap < c.nvals + nv[i]) cap *= 2;
          DevBuf bigger(m->ctx, size_t(cap) * 4);
          if (c.nvals)
            hip_check(hipMemcpyAsync(bigger.p, c.ids.p, size_t(c.nvals) * 4, hipMemcpyDeviceToDevice, st), "grow");
          hip_check(hipStreamSynchronize(st), "sync");
          c.ids = std::move(bigger);
          c.ids_cap = cap;
        }
      }
      const int64_t at = c.mv ? c.nvals : m->num_docs;
      hip_check(hipMemcpyAsync(c.ids.as<int32_t>() + at, ids[i], size_t(nv[i]) * 4, hipMemcpyHostToDevice, st),
                "ids H2D");
    }
    hip_check(hipStreamSynchronize(st), "sync");  // the caller's buffers may go away after the call
    for (size_t i = 0; i < ncols; ++i) {  // commit: every column was accepted
      pgx_mutable::Col& c = m->cols[i];
      c.max_id = std::max(c.max_id, top[i]);
      if (c.mv) {
        c.nvals += nv[i];
        c.max_mv = std::max(c.max_mv, mvmax[i]);
      }
    }
    m->num_docs += ndocs;
  });
}

pgx_status pgx_mutable_set_dictionary(pgx_mutable* m, int32_t col, int32_t card, const void* dict, uint64_t dict_len,
                                      int32_t dict_width, int32_t pad_char, const int32_t* arrival_to_sorted) {
  return guarded([&] {
    if (!m || !dict || !arrival_to_sorted || card < 1) fail(PGX_ERR_INVALID_ARG, "bad argument");
    std::lock_guard<std::mutex> g(m->mu);
    if (col < 0 || col >= int(m->cols.size())) fail(PGX_ERR_INVALID_ARG, "column index");
    pgx_mutable::Col& c = m->cols[col];
    const int width = (c.data_type == PGX_INT || c.data_type == PGX_FLOAT) ? 4 : c.data_type == PGX_STRING ? dict_width : 8;
    if (width < 1 || dict_len < uint64_t(width) * card) fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": dictionary short");
    for (int32_t i = 0; i < card; ++i)
      if (arrival_to_sorted[i] < 0 || arrival_to_sorted[i] >= card)
        fail(PGX_ERR_INVALID_ARG, "column " + c.name + ": remap out of range");
    hip_check(hipSetDevice(m->ctx->device), "hipSetDevice");
    c.card = card;
    c.dict_width = width;
    c.pad_char = pad_char & 0xFF;
    c.dict.assign(static_cast<const uint8_t*>(dict), static_cast<const uint8_t*>(dict) + uint64_t(width) * card);
    c.remap = DevBuf(m->ctx, size_t(card) * 4);
    hip_check(hipMemcpy(c.remap.p, arrival_to_sorted, size_t(card) * 4, hipMemcpyHostToDevice), "remap H2D");
  });
}

pgx_status pgx_mutable_snapshot(pgx_mutable* m, pgx_segment** out) {
  return guarded([&] {
    if (!m || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> g(m->mu);
    if (m->num_docs < 1) fail(PGX_ERR_INVALID_ARG, "realtime segment " + m->name + " has no docs");
    pgx_ctx* ctx = m->ctx;
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = ctx->stream;
    auto seg = std::make_unique<pgx_segment>();
    seg->ctx = ctx;
    seg->name = m->name;
    seg->total_docs = seg->total_raw_docs = m->num_docs;
    seg->cols.resize(m->cols.size());
    const int64_t n = m->num_docs;
    for (size_t i = 0; i < m->cols.size(); ++i) {
      const pgx_mutable::Col& mc = m->cols[i];
      StagedColumn& c = seg->cols[i];
      if (mc.card < 1 || mc.max_id >= mc.card)
        fail(PGX_ERR_INVALID_ARG, "column " + mc.name + ": dictionary not set for every appended value");
      c.name = mc.name;
      c.data_type = mc.data_type;
      c.card = mc.card;
      c.bits = bits_for(mc.card);
      c.dict_width = mc.dict_width;
      c.pad_char = mc.pad_char;
      c.is_sorted = false;           // RealtimeColumnDataSource.isSorted(): false
      c.has_inverted = mc.inverted;  // bitmap-filter semantics; without index bytes the leaf is evaluated by scanning
      stage_dict(ctx, seg.get(), mc.dict, c);
      const int64_t rows = mc.mv ? mc.nvals : n;
      const uint64_t need = padded_fwd_bytes(rows, c.bits);
      c.fwd_owned = DevBuf(ctx, need);
      hip_check(hipMemsetAsync(c.fwd_owned.p, 0, need, st), "memset");
      PGX_LAUNCH(st, "pgx_pack_remap", pgx_launch_pack_remap(c.fwd_owned.as<uint32_t>(), mc.ids.as<int32_t>(),
                                                              mc.remap.as<int32_t>(), rows, c.bits,
                                                              int64_t((uint64_t(rows) * c.bits + 31) / 32), st),
                 "realtime forward index");
      c.fwd = c.fwd_owned.as<const uint32_t>();
      seg->device_bytes += need;
      if (mc.mv) {
        c.is_mv = true;
        c.total_entries = mc.nvals;
        c.max_mv = mc.max_mv;
        c.mv_start = DevBuf(ctx, (size_t(n) + 1) * 4);
        hip_check(hipMemcpyAsync(c.mv_start.p, mc.starts.p, (size_t(n) + 1) * 4, hipMemcpyDeviceToDevice, st),
                  "starts copy");
        seg->device_bytes += (size_t(n) + 1) * 4;
      }
      seg->by_name[c.name] = int(i);
      seg->names.push_back(c.name);
    }
    hip_check(hipStreamSynchronize(st), "sync");
    ctx->refs.fetch_add(1);  // released by pgx_segment_release
    *out = seg.release();
  });
}

pgx_status pgx_mutable_num_docs(const pgx_mutable* m, int32_t* out) {
  return guarded([&] {
    if (!m || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    std::lock_guard<std::mutex> g(m->mu);  // appends write num_docs under the same lock
    *out = m->num_docs;
  });
}

pgx_status pgx_mutable_release(pgx_mutable* m) {
  return guarded([&] {
    if (!m) return;
    pgx_ctx* ctx = m->ctx;
    delete m;
    if (ctx) ctx_unref(ctx);
  });
}

}  // extern "C"
