// libpgx host side: the C ABI of include/pgx.h.
//
// Segment staging (Loaders / ColumnIndexContainer), per-query physical planning (FilterPlanNode's operator choice,
// the AND/OR algebra as a postfix program, DefaultGroupKeyGenerator's key space), launch of the fused HIP kernel and
// decoding of the combined result (MCombine*Operator + AggregationGroupByOperatorService.trimToSize).  The partitioned
// sparse group-by runtime is pgx_part.cpp; the shared types are pgx_host.h.
// Reference paths are relative to pinot-core/src/main/java/com/linkedin/pinot/core/.
#include "pgx_host.h"


namespace pgxh {
size_t align_up(size_t x, size_t a) { return (x + a - 1) & ~(a - 1); }

// Bitmap inverted-index leaves: one mask per (segment, leaf) (pgx_roaring_expand), or one mask per (segment, bitmap
// program) with the sub-tree's AND / OR / NOT applied in the same pass (pgx_roaring_program).
// Bitmap programs are pure mask algebra (the statistics come from the filter tree, not from here), so AND's operands
// commute: an AND whose left operand is NOT(leaf) gets it as its right operand instead, which turns
// "NOT c, (a OR b), AND" into "(a OR b), c, NOT, AND": the form the wave kernel folds into one mask slot (AND-NOT).
void canon_rprog(std::vector<int>& op, std::vector<int>& arg) {
  struct Node { int op, arg, l, r; };
  std::vector<Node> nodes;
  std::vector<int> st;
  for (size_t i = 0; i < op.size(); ++i) {
    Node nd{op[i], arg[i], -1, -1};
    if (op[i] == RP_NOT) {
      if (st.empty()) return;  // malformed: leave as is
      nd.l = st.back();
      st.pop_back();
    } else if (op[i] != RP_LEAF) {
      if (st.size() < 2) return;
      nd.r = st.back();
      st.pop_back();
      nd.l = st.back();
      st.pop_back();
    }
    nodes.push_back(nd);
    st.push_back(int(nodes.size()) - 1);
  }
  if (st.size() != 1) return;
  auto neg_leaf = [&](int x) { return nodes[x].op == RP_NOT && nodes[nodes[x].l].op == RP_LEAF; };
  std::vector<int> o2, a2;
  std::function<void(int)> out = [&](int x) {
    const Node& nd = nodes[x];
    if (nd.op == RP_NOT) {
      out(nd.l);
    } else if (nd.op != RP_LEAF) {
      const bool swap = nd.op == RP_AND && neg_leaf(nd.l) && !neg_leaf(nd.r);
      out(swap ? nd.r : nd.l);
      out(swap ? nd.l : nd.r);
    }
    o2.push_back(nd.op);
    a2.push_back(nd.arg);
  };
  out(st[0]);
  op.swap(o2);
  arg.swap(a2);
}

// Mask slots the wave-per-chunk kernel (pgx_roaring_program_wave) needs for one program.  While the top operand is
// "pure" (an OR of leaves, nothing applied yet), a leaf directly followed by OR is ORed into its slot, and a leaf
// directly followed by NOT, AND is cleared out of it (which ends its purity); every other leaf takes a new slot.
int rprog_slots(const RProg& r) {
  std::vector<bool> pure;  // the operand stack's "pure OR of leaves" flags
  int ns = 0;
  for (int i = 0; i < r.nops; ++i) {
    const int op = r.op[i];
    if (op == RP_LEAF) {
      const bool top = !pure.empty() && pure.back();
      const bool f_or = top && i + 1 < r.nops && r.op[i + 1] == RP_OR;
      const bool f_andnot = top && !f_or && i + 2 < r.nops && r.op[i + 1] == RP_NOT && r.op[i + 2] == RP_AND;
      if (f_or) {
        ++i;
      } else if (f_andnot) {
        pure.back() = false;
        i += 2;
      } else {
        pure.push_back(true);
        ++ns;
      }
    } else if (op == RP_NOT) {
      if (!pure.empty()) pure.back() = false;
    } else if (pure.size() >= 2) {
      pure.pop_back();
      pure.back() = false;
    }
  }
  return ns;
}

// The wave kernel's own plan walk (pgx_roaring_program_wave) keeps the operand stack as 4-bit entries of one 64-bit
// word and shifts on every binary op unconditionally: only well-formed programs (each NOT / AND / OR has its operands,
// one result left), at most 16 operands deep and with slot ids below 8 may take it.  Mirrors the device walk.
bool rprog_wave_ok(const RProg& r, int* slots) {
  int depth = 0, maxd = 0, ns = 0;
  std::vector<bool> pure;
  for (int i = 0; i < r.nops; ++i) {
    const int op = r.op[i];
    if (op == RP_LEAF) {
      const bool top = !pure.empty() && pure.back();
      const bool f_or = top && i + 1 < r.nops && r.op[i + 1] == RP_OR;
      const bool f_andnot = top && !f_or && i + 2 < r.nops && r.op[i + 1] == RP_NOT && r.op[i + 2] == RP_AND;
      if (f_or) {
        ++i;
      } else if (f_andnot) {
        pure.back() = false;
        i += 2;
      } else {
        pure.push_back(true);
        ++ns;
        maxd = std::max(maxd, ++depth);
      }
    } else if (op == RP_NOT) {
      if (depth < 1) return false;
      pure.back() = false;
    } else if (op == RP_AND || op == RP_OR) {
      if (depth < 2) return false;
      --depth;
      pure.pop_back();
      pure.back() = false;
    } else {
      return false;
    }
  }
  if (depth != 1 || maxd > 16 || ns > 7) return false;
  if (slots) *slots = ns;
  return true;
}

// Bitmap programs [p0, p1) (default: all of them).
void launch_bitmaps(ExecPlan& P, hipStream_t st, int p0 = 0, int p1 = -1) {
  if (P.rchunk) return;  // the query kernels evaluate the bitmap programs per chunk themselves
  if (P.rprog_on) {
    if (p1 < 0) p1 = int(P.rprogs.size());
    const int np = p1 - p0;
    const RProg* progs = P.rprog_dev + p0;
    if (P.rp_kind < 0) {  // once per plan: the choice depends on the programs only
      // wave-per-chunk kernel when every program has <= 64 bitmaps (one lane each) and <= 3 mask slots
      const int rk = P.kn.rprog;  // PGX_RPROG: wave | seg | chunk | stack (default: the first that fits)
      bool wave = rk == RPROG_AUTO || rk == RPROG_WAVE;
      int nslots = 1;
      for (size_t i = 0; i < P.rprogs.size() && wave; ++i) {
        const RProg& r = P.rprogs[i];
        int nb = 0;
        for (int k = 0; k < r.nops; ++k)
          if (r.op[k] == RP_LEAF && r.arg[k] >= 0) nb += P.roar[r.arg[k]].nb;
        int ns = 0;
        if (!rprog_wave_ok(r, &ns) || ns != rprog_slots(r)) wave = false;
        if (nb > 64 || ns > 3) wave = false;
        nslots = std::max(nslots, ns);
      }
      int maxleaves = 0;  // leaf masks the wide kernel keeps in LDS (PGX_RPROG=stack: the stack kernel)
      if (!wave) {
        for (const auto& dp : P.dm_progs) {
          int nl = 0;
          for (int8_t o : dp.op) nl += o == RP_LEAF;
          maxleaves = std::max(maxleaves, nl);
        }
        if (rk == RPROG_STACK) maxleaves = 0;
        // per-segment container walk when every program's bitmaps fit one lane each (PGX_RPROG=chunk: per-chunk kernels)
        bool seg_walk = maxleaves >= 1 && rk != RPROG_CHUNK && rk != RPROG_STACK;
        for (size_t i = 0; i < P.rprogs.size() && seg_walk; ++i) {
          int nb = 0;
          const RProg& r = P.rprogs[i];
          for (int k = 0; k < r.nops; ++k)
            if (r.op[k] == RP_LEAF && r.arg[k] >= 0) nb += P.roar[r.arg[k]].nb;
          if (nb > 512) seg_walk = false;
        }
        if (seg_walk) maxleaves = -maxleaves;
      }
      P.rp_kind = wave ? 0 : 1;
      P.rp_nslots = nslots;
      P.rp_maxleaves = maxleaves;
    }
    if (P.rp_kind == 0) {
      PGX_LAUNCH(st, "pgx_roaring_program_wave", pgx_launch_roaring_program_wave(progs, P.rdesc_dev, np, P.roar_maxchunks, P.rp_nslots, st),
                "bitmap program launch");
      return;
    }
    PGX_LAUNCH(st, "pgx_roaring_program", pgx_launch_roaring_program(progs, P.rdesc_dev, np, P.roar_maxchunks, P.rp_maxleaves, st),
              "bitmap program launch");
  } else if (P.rdesc_dev) {
    PGX_LAUNCH(st, "pgx_roaring", pgx_launch_roaring(P.rdesc_dev, int(P.roar.size()), P.roar_maxchunks, st), "bitmap expansion launch");
  }
}

// Host half of the argument upload: lays out and fills the pinned arena (blob, KSeg, RDesc, RProg) and allocates the
// device buffers the plan needs.  No stream work: batched plans build their arenas on planner threads.
void build_arena(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B) {
  const size_t n = P.ksegs.size();
  B.off_ksegs = align_up(P.blob32.size() * 4, 256);
  B.off_jsegs = align_up(B.off_ksegs + n * sizeof(KSeg), 256);
  P.star_tile_cap = 0;
  for (int s = 0; s < int(n); ++s)
    // tiles of at least 256 threads x 8 rows (plan_jit may shrink rows per lane per tile to 8 for wide queries)
    if (!P.star.empty() && P.star[s].on) P.star_tile_cap += size_t(P.ksegs[s].num_docs) / 2048 + 2;
  B.off_tiles = align_up(B.off_jsegs + n * sizeof(JSeg), 256);
  B.off_rdesc = align_up(B.off_tiles + P.star_tile_cap * 4, 256);
  B.off_rprog = align_up(B.off_rdesc + P.roar.size() * sizeof(RDesc), 256);
  B.off_outs = align_up(B.off_rprog + P.rprogs.size() * sizeof(RProg), 256);
  const KQuery& K0 = P.kq;
  const uint64_t tbl = (K0.group_mode == G_DENSE_LDS || K0.group_mode == G_DENSE_GLOBAL) && !P.use_part
                           ? P.dense_slots * uint64_t(K0.num_planes) * 8
                           : 0;
  B.tbl_bytes = tbl <= kArenaTableMax ? size_t(tbl) : 0;
  B.tbl_live = false;
  B.size = B.off_outs + kOutsBytes + B.tbl_bytes;
  B.arena = DevBuf(ctx, B.size);
  B.host = PinnedBuf(ctx, B.size);
  if (!P.blob32.empty()) std::memcpy(B.host.bytes(), P.blob32.data(), P.blob32.size() * 4);
  const int32_t* base = reinterpret_cast<const int32_t*>(B.dev());
  for (const auto& f : P.fixes) {
    KSeg& S = P.ksegs[f.seg];
    if (f.kind == 0) S.remap[f.slot] = base + f.off;
    else if (f.kind == 1) S.leaf[f.slot].ranges = base + f.off;
    else S.leaf[f.slot].bitset = reinterpret_cast<const uint32_t*>(base + f.off);
  }
  P.lmask_dev = nullptr;
  if (P.fsm_on) {
    const int S = P.fsm.num_states;
    P.lmask_buf = DevBuf(ctx, std::max<uint64_t>(P.lmask_total, 1) * 4);
    P.lmask_dev = P.lmask_buf.as<uint32_t>();
    size_t fi = 0;
    for (size_t s = 0; s < n; ++s) {
      if (P.lmask_off[s] < 0) continue;
      P.ksegs[s].lmask = P.lmask_dev + P.lmask_off[s];
      P.ksegs[s].lmask_words = P.lmask_words[s];
      P.fsm_segs[fi++].lmask = P.lmask_dev + P.lmask_off[s];
    }
    P.fsm_table = DevBuf(ctx, P.fsm.table.size() * 4);
    P.fsm_segbuf = DevBuf(ctx, P.fsm_segs.size() * sizeof(FsmSeg));
    const uint64_t ent = std::max<uint64_t>(uint64_t(P.fsm_chunks) * S, 1);
    P.fsm_cnt = DevBuf(ctx, ent * 4);
    P.fsm_stv = DevBuf(ctx, ent * 2);
    P.fsm_T = std::max(1, std::min(64, 512 / S));
    const uint64_t pe = uint64_t(P.fsm_segs.size()) * P.fsm_T * S;
    P.fsm_pcount = DevBuf(ctx, pe * 8);
    P.fsm_pstate = DevBuf(ctx, pe * 2);
  }
  P.mv_host.clear();
  if (!P.mv_items.empty()) {  // multi-value scan leaves: descriptors + one doc mask per (segment, leaf)
    std::vector<MvLeaf>& items = P.mv_host;
    items.resize(P.mv_items.size());
    std::vector<int64_t> off(P.mv_items.size());
    int64_t words = 0;
    P.mv_max_words = 0;
    for (size_t i = 0; i < items.size(); ++i) {
      const int w = (P.ksegs[P.mv_items[i].seg].num_docs + 31) / 32 + 1;
      off[i] = words;
      words += w;
      P.mv_max_words = std::max(P.mv_max_words, w);
    }
    P.mv_masks = DevBuf(ctx, size_t(std::max<int64_t>(words, 1)) * 4);
    for (size_t i = 0; i < items.size(); ++i) {
      const auto& it = P.mv_items[i];
      const KSeg& S = P.ksegs[it.seg];
      const KLeaf& L = S.leaf[it.leaf];
      const StagedColumn& col = *P.segcols[it.seg][P.kq.leaf_col[it.leaf]];
      MvLeaf& m = items[i];
      m.vals = col.fwd;
      m.start = col.mv_start.as<const int32_t>();
      m.bitset = L.mode == LEAF_SCAN_BITSET ? L.bitset : nullptr;
      m.mask = P.mv_masks.as<uint32_t>() + off[i];
      m.bits = col.bits;
      m.num_docs = S.num_docs;
      m.lo = uint32_t(L.lo);
      m.span = uint32_t(L.hi) - uint32_t(L.lo);
      m.neg = P.mv_neg.empty() ? 0 : P.mv_neg[it.leaf];
      P.ksegs[it.seg].leaf[it.leaf].bitset = m.mask;  // the query kernel's LEAF_DOCMASK word source
    }
    P.mv_descs = DevBuf(ctx, items.size() * sizeof(MvLeaf));
  }
  if (n) std::memcpy(B.host.bytes() + B.off_ksegs, P.ksegs.data(), n * sizeof(KSeg));
  P.kq.segs = reinterpret_cast<const KSeg*>(B.dev() + B.off_ksegs);
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.dev() + B.off_outs);
  P.kq.agg_out = outs;
  P.kq.stats = outs + 16;
  P.kq.overflow = outs + 24;
  // bitmap inverted-index expansion descriptors + the per-(segment, leaf) doc masks they fill
  P.rdesc_dev = nullptr;
  P.masks_dev = nullptr;
  P.rprog_dev = nullptr;
  if (!P.roar.empty() || !P.rprogs.empty()) {
    B.masks = DevBuf(ctx, std::max<uint64_t>(P.mask_words, 1) * 4);
    P.masks_dev = B.masks.as<uint32_t>();
    RDesc* rd = reinterpret_cast<RDesc*>(B.host.bytes() + B.off_rdesc);
    for (size_t i = 0; i < P.roar.size(); ++i) {
      const auto& it = P.roar[i];
      rd[i].mask = P.rprog_on ? nullptr : P.masks_dev + it.mask_off;
      rd[i].inv = static_cast<const uint8_t*>(it.inv);
      rd[i].ids = reinterpret_cast<const uint32_t*>(base + it.blob_off);
      rd[i].nb = it.nb;
      rd[i].nchunks = it.nchunks;
    }
    P.rdesc_dev = reinterpret_cast<const RDesc*>(B.dev() + B.off_rdesc);
    RProg* rp = reinterpret_cast<RProg*>(B.host.bytes() + B.off_rprog);
    for (size_t i = 0; i < P.rprogs.size(); ++i) {
      rp[i] = P.rprogs[i];
      rp[i].mask = P.masks_dev + uintptr_t(P.rprogs[i].mask);  // word offset -> device pointer
    }
    P.rprog_dev = reinterpret_cast<const RProg*>(B.dev() + B.off_rprog);
  }
}

// Stream half: the automaton / multi-value descriptor copies, and -- so the bitmap expansion runs on the GPU while the
// host plans the query kernels (plan_jit) -- the blob (roaring offsets) and bitmap descriptors ahead of the rest of the
// arena, then the bitmap launch.
void send_arena(ExecPlan& P, ExecBuffers& B, hipStream_t st) {
  if (P.fsm_on) {
    hip_check(hipMemcpyAsync(P.fsm_table.p, P.fsm.table.data(), P.fsm.table.size() * 4, hipMemcpyHostToDevice, st),
              "automaton tables H2D");
    hip_check(hipMemcpyAsync(P.fsm_segbuf.p, P.fsm_segs.data(), P.fsm_segs.size() * sizeof(FsmSeg),
                             hipMemcpyHostToDevice, st),
              "automaton segments H2D");
  }
  if (!P.mv_host.empty())  // pageable source: the copy completes before the call returns (P keeps it alive anyway)
    hip_check(hipMemcpyAsync(P.mv_descs.p, P.mv_host.data(), P.mv_host.size() * sizeof(MvLeaf), hipMemcpyHostToDevice,
                             st),
              "multi-value leaf descriptors H2D");
  if (P.rdesc_dev || P.rprog_dev) {
    hip_check(hipMemcpyAsync(B.arena.p, B.host.p, P.blob32.size() * 4, hipMemcpyHostToDevice, st), "blob H2D");
    hip_check(hipMemcpyAsync(B.dev() + B.off_rdesc, B.host.bytes() + B.off_rdesc,
                             B.off_outs - B.off_rdesc, hipMemcpyHostToDevice, st), "bitmap descriptors H2D");
    launch_bitmaps(P, st);
    P.roar_early = !P.rchunk;
  }
}

void upload_plan(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, hipStream_t st) {
  build_arena(ctx, P, B);
  send_arena(P, B, st);
}

void alloc_outputs(pgx_ctx* ctx, ExecPlan& P, ExecBuffers& B, void* dense_out, uint64_t dense_out_bytes) {
  KQuery& K = P.kq;
  K.table = nullptr;
  K.keys = nullptr;
  K.key_state = nullptr;
  B.tbl_live = false;
  if (K.group_mode == G_DENSE_LDS || K.group_mode == G_DENSE_GLOBAL) {
    K.dense_slots = P.dense_slots;
    const uint64_t bytes = P.dense_slots * K.num_planes * 8;
    if (dense_out) {
      if (dense_out_bytes < bytes) fail(PGX_ERR_INVALID_ARG, "dense_out too small");
      K.table = static_cast<unsigned long long*>(dense_out);
    } else if (bytes && B.tbl_bytes == bytes) {
      K.table = reinterpret_cast<unsigned long long*>(B.dev() + B.off_outs + kOutsBytes);
      B.tbl_live = true;
    } else {
      if (!B.table.p || B.table_bytes != bytes) {  // (a kept plan reuses its table: clean after a resetting compaction)
        B.table = DevBuf(ctx, bytes);
        B.table_bytes = bytes;
        B.table_clean = false;
      }
      K.table = devp(B.table);
    }
  } else if (P.use_part && !P.part_slab) {
    B.table_bytes = 0;
    B.table_clean = false;
    B.table = DevBuf(ctx, std::max<int64_t>(P.rec_total, 1) * 8);  // one key|value record per scanned row
    K.table = devp(B.table);
  } else if (hash_mode(K.group_mode)) {
    K.hash_cap = P.hash_cap;
    B.table_bytes = 0;
    B.table_clean = false;
    B.table = DevBuf(ctx, P.hash_cap * K.num_planes * 8);
    K.table = devp(B.table);
    const uint64_t kw = uint64_t(K.key_words) * P.hash_cap;
    B.keys = DevBuf(ctx, kw * 8);
    K.keys = devp(B.keys);
    if (K.group_mode != G_HASH64) {
      B.key_state = DevBuf(ctx, P.hash_cap * 4);
      K.key_state = B.key_state.as<unsigned int>();
    }
  }
}

void reset_outputs(ExecPlan& P, ExecBuffers& B, hipStream_t st, bool init_table, bool outs_only) {
  // (re)sends the whole argument arena with initialised output planes; outs_only: the arena's descriptors are already
  // on the device (a cached plan's replay: kernels write only the outputs block), send the outputs block alone
  KQuery& K = P.kq;
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
  std::memset(outs, 0, kOutsBytes);
  for (int p = 1; p < K.num_planes; ++p) outs[p] = (K.plane_op[p] == P_MIN_ORD) ? ~0ull : 0ull;
  const bool tbl = B.tbl_live && init_table;  // the in-arena dense table travels with the outputs block
  if (tbl) {
    unsigned long long* t = outs + kOutsBytes / 8;
    const uint64_t slots = P.dense_slots;
    for (int p = 0; p < K.num_planes; ++p)
      std::fill(t + p * slots, t + (p + 1) * slots, (K.plane_op[p] == P_MIN_ORD) ? ~0ull : 0ull);
  }
  if (outs_only)
    hip_check(hipMemcpyAsync(B.dev() + B.off_outs, outs, kOutsBytes + (tbl ? B.tbl_bytes : 0), hipMemcpyHostToDevice,
                             st),
              "outputs H2D");
  else
    hip_check(hipMemcpyAsync(B.arena.p, B.host.p, B.size, hipMemcpyHostToDevice, st), "argument arena H2D");
  if (init_table && K.group_mode != G_NONE && !P.use_part && !B.tbl_live) {
    const uint64_t slots = hash_mode(K.group_mode) ? P.hash_cap : P.dense_slots;
    const uint64_t kw = hash_mode(K.group_mode) ? uint64_t(K.key_words) * P.hash_cap : 0;
    const bool clean = !hash_mode(K.group_mode) && B.table_clean && B.table.p && K.table == devp(B.table);
    if (!clean)
      PGX_LAUNCH(st, "pgx_init_planes", pgx_launch_init_planes(K.table, slots, K.num_planes, &K, K.keys, kw, K.key_state, st), "init planes");
    B.table_clean = false;  // this execution's kernels accumulate into it
  }
}

// Build the query-specialised launch groups (pgx_jit.cpp) for plans the generated kernels cover: aggregation-only
// and dense group-by over at most PGX_J_MAX_COLS columns.  Hash group-by keeps the generic kernel.  PGX_JIT=0 forces
// the generic kernel (A/B timing); both are HIP paths with identical accumulator encodings.

// Workgroups of a generated kernel resident per CU (LDS, registers, waves), cached per kernel.  The persistent grids
// are sized to exactly one round: a second, partial round of workgroups would run the tail at a fraction of the chip.
int jit_occupancy(void* fn, int threads) {
  static std::mutex mu;
  static std::map<void*, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(fn);
  if (it != cache.end()) return it->second;
  int occ = 0;
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&occ, static_cast<hipFunction_t>(fn), threads, 0) !=
          hipSuccess || occ < 1)
    occ = 1;
  cache.emplace(fn, occ);
  return occ;
}

void plan_jit(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, ExecPlan& P, ExecBuffers& B) {
  P.jit.clear();
  P.part_nwg = 0;
  P.part_wg_rows = 0;
  const bool slab = P.part_slab;
  P.part_slab = false;  // only the query kernels write slabs (the generic kernel writes row-order records)
  const KQuery& K = P.kq;
  if (!P.kn.jit) return;
  if (!(K.group_mode == G_NONE || K.group_mode == G_DENSE_LDS || K.group_mode == G_DENSE_GLOBAL || P.use_part ||
        K.group_mode == G_HASH64 || K.group_mode == G_HASH128))
    return;  // (G_HASHW: keys of 3-4 words stay on the generic kernel)
  const int nc = K.num_qcols;
  if (nc > PGX_J_MAX_COLS) return;
  P.part_slab = slab;
  const bool grouped = K.group_mode != G_NONE;
  // which columns are decoded, which carry value images
  std::vector<bool> decode(nc, false), want_img(nc, false);
  const int nleaves = int(q.leaf_col.size());
  for (int a = 0; a < K.num_aggs; ++a) {
    if (K.agg_kind[a] == A_COUNT) continue;
    decode[K.agg_col[a]] = true;
    if (grouped || K.agg_kind[a] == A_SUM || K.agg_kind[a] == A_AVG) want_img[K.agg_col[a]] = !P.part_dictid;
  }
  for (int g = 0; g < K.num_gcols; ++g) decode[K.gcol[g]] = true;
  // signature per segment -> groups (a flat int vector per segment, compared whole; one std::map lookup each)
  std::map<std::vector<int32_t>, std::vector<int>> groups;
  std::vector<const std::vector<int32_t>*> order;
  std::vector<int32_t> sig;
  for (int s = 0; s < n; ++s) {
    const KSeg& S = P.ksegs[s];
    sig.clear();
    for (int l = 0; l < nleaves; ++l)
      sig.push_back(P.roar_index[s][l] >= 0 ? (P.roar[P.roar_index[s][l]].neg ? 101 : 100)
                                            : (P.mv_index[s][l] >= 0 ? 102 : S.leaf[l].mode));
    if (P.star[s].on) {
      sig.push_back(-7);
      for (size_t i = 0; i < P.star[s].op.size(); ++i) {
        sig.push_back(P.star[s].op[i]);
        sig.push_back(P.star[s].arg[i]);
      }
    }
    sig.push_back(-1);
    for (int c = 0; c < nc; ++c) {
      const StagedColumn& col = *P.segcols[s][c];
      sig.push_back(S.bits[c] | (S.remap[c] ? 256 : 0));
      if (want_img[c]) sig.push_back(col.img_kind * 64 + col.img_sh);
    }
    auto it = groups.find(sig);
    if (it == groups.end()) {
      it = groups.emplace(sig, std::vector<int>{}).first;
      order.push_back(&it->first);
    }
    it->second.push_back(s);
  }
  prof_mark("j.sig");
  const int cus = ctx->num_cus;
  size_t jidx = 0;  // next free JSeg slot of the arena
  size_t star_tile_off = 0;
  P.star_tiles.assign(n, {});
  for (const std::vector<int32_t>* key : order) {
    const std::vector<int>& members = groups[*key];
    const KSeg& S0 = P.ksegs[members[0]];
    JitShape J;
    J.cols.resize(nc);
    std::vector<bool> dec = decode;
    for (int l = 0; l < nleaves; ++l)
      if ((S0.leaf[l].mode == LEAF_SCAN_INTERVAL || S0.leaf[l].mode == LEAF_SCAN_BITSET) &&
          P.roar_index[members[0]][l] < 0 && P.mv_index[members[0]][l] < 0)
        dec[K.leaf_col[l]] = true;
    int R = 8;
    for (int c = 0; c < nc; ++c) {
      JitCol& C = J.cols[c];
      C.bits = S0.bits[c];
      C.decode = dec[c];
      C.remap = S0.remap[c] != nullptr;
      const StagedColumn& col0 = segs[members[0]]->col(P.qcols[c]);
      C.fp = col0.data_type == PGX_FLOAT || col0.data_type == PGX_DOUBLE;
      if (C.decode) {
        int g = 1;
        while (g < 32 && (C.bits % (g * 2)) == 0) g *= 2;  // largest power of two dividing bits (<= 32)
        R = std::max(R, 32 / g);
      }
      if (want_img[c]) {
        C.img = col0.img_kind;
        C.img_sh = col0.img_sh;
        uint64_t range = 0;
        for (int s : members) {
          const StagedColumn& col = *P.segcols[s][c];
          C.img_words = std::max(C.img_words, col.img_words);
          range = std::max(range, col.vrange);
        }
        C.acc32 = range * 32 < 0xFFFFFFFFull;
      }
    }
    J.R = R;
    // Registers for the raw words of the next tile (loaded one tile ahead, so held twice): sum over the decoded columns
    // of the dwords one sub-step of R rows takes, times the sub-steps per tile.  A query over many columns (C6: twelve)
    // at 32 rows per lane per tile needs ~250 VGPRs for them alone and spills at the 1024-thread workgroups an LDS image
    // asks for: take eight rows per lane (fractional loads of odd widths) and fewer rows per lane per tile until the
    // double-buffered words fit kTileWordBudget.  C2 / C5 shapes (two or three columns) keep 32 rows per lane per tile.
    {
      constexpr int kTileWordBudget = 64;
      auto words = [&](int r) {
        int w = 0;
        for (const JitCol& C : J.cols) {
          if (!C.decode) continue;
          const int rb = r * C.bits;
          if (rb % 32 == 0) {
            w += rb / 32;
          } else {
            int g = 32;
            while (rb % g) g >>= 1;
            w += (rb + 32 - g + 31) / 32;
          }
        }
        return w;
      };
      if (J.R > 8 && 2 * words(J.R) > kTileWordBudget) {
        J.R = 8;
        for (JitCol& C : J.cols) C.frac = C.decode && (8 * C.bits) % 32 != 0;
      }
      const int w = words(J.R);
      while (J.TL > J.R && 2 * (J.TL / J.R) * w > kTileWordBudget) J.TL /= 2;
    }
    if (P.kn.no_img && !P.use_part)
      for (JitCol& C : J.cols) C.img = IMG_NONE;
    // LDS budget: drop the largest images until everything fits (LEAF_RCHUNK: a budget for three workgroups per CU)
    int64_t rch_bytes = 0;
    if (P.rchunk) {
      const size_t np = P.dm_progs.size();
      for (size_t k = 0; k < np; ++k) {
        const RProg& r0 = P.rprogs[size_t(members[0]) * np + k];
        std::vector<int> ops(r0.op, r0.op + r0.nops);
        int nl = 0;
        for (int op : ops) nl += op == RP_LEAF;
        if (nl > PGX_J_MAX_RLEAVES) fail(PGX_ERR_UNSUPPORTED, "bitmap program with too many leaves");
        rch_bytes += int64_t(nl) * 8192;
        J.rprog_ops.push_back(std::move(ops));
      }
      rch_bytes += 5152;  // container-search scratch
    }
    const int64_t lds_budget = P.rchunk ? 52 * 1024 : kLdsBudget;
    // hash group-by: the workgroup's LDS table (keys, 128-bit key states, planes); 2048 slots when they fit beside the
    // images, down to 512 before an image is dropped
    const bool hashg = K.group_mode == G_HASH64 || K.group_mode == G_HASH128;
    // a packed count + sum table (COUNT + one integer SUM / AVG over an image: dense_pack below, pgx_jit.cpp hpack)
    // holds one plane per slot: 4096 slots then fit beside a 16 KiB image (load 1/4 at C7's 1024 groups: shorter probes)
    bool hp1 = hashg && K.num_planes == 2 && K.num_aggs == 1 && (K.agg_kind[0] == A_SUM || K.agg_kind[0] == A_AVG) &&
               K.agg_col[0] >= 0 && !K.agg_fp[0] && J.cols[K.agg_col[0]].img != IMG_NONE;
    auto hslot_bytes = [&]() -> int64_t {
      return hashg ? (K.group_mode == G_HASH128 ? 20 : 8) + 8 * (hp1 ? 1 : K.num_planes) : 0;
    };
    int hash_slots = hashg ? (hp1 ? 4096 : 2048) : 0;
    auto lds_need = [&]() {
      int64_t b = rch_bytes + (hashg ? hash_slots * hslot_bytes() + 32 : 0);
      for (const JitCol& C : J.cols)
        if (C.img != IMG_NONE) b += ((int64_t(C.img_words) * 4 + 15) / 16) * 16;
      if (K.group_mode == G_DENSE_LDS) b += int64_t(P.dense_slots) * K.num_planes * 8;
      return b;
    };
    while (hashg && hash_slots > 512 && lds_need() > lds_budget) hash_slots /= 2;
    while (lds_need() > lds_budget) {
      int big = -1;
      for (int c = 0; c < nc; ++c)
        if (J.cols[c].img != IMG_NONE && (big < 0 || J.cols[c].img_words > J.cols[big].img_words)) big = c;
      if (big < 0) {
        if (P.rchunk) fail(PGX_ERR_INTERNAL, "bitmap-program kernel LDS budget");
        return;  // the dense LDS table alone does not fit: generic kernel
      }
      J.cols[big].img = IMG_NONE;
    }
    if (hp1 && J.cols[K.agg_col[0]].img == IMG_NONE) {  // the image went: no packed table, two planes per slot
      hp1 = false;
      while (hash_slots > 512 && lds_need() > lds_budget) hash_slots /= 2;
    }
    const int64_t lds = lds_need();
    J.T = lds <= 20 * 1024 ? 256 : (lds <= 40 * 1024 ? 512 : 1024);
    if (P.rchunk) J.T = 512;  // three 512-thread workgroups per CU, four tiles per chunk
    if (P.use_part) J.T = std::min(J.T, 512);  // record-emitting kernels hold R 64-bit records per lane: 256 VGPRs
    if (P.part_narrow) {
      // the narrow split's LDS rings (pgx_jit.cpp) want ~16 records per bucket per sub-step (T * R = 4096: a ring of
      // 64 holds the unflushed unit plus the sub-step's records with a wide margin): 512 threads, eight rows per lane
      // (fractional loads of widths that need it), half tiles (16 rows per lane) so the raw words of the next tile stay
      // in registers without spilling (1024 threads and 16 or 32 rows per lane measured slower).
      // (PGX_DEBUG nunit=16: 16-record units in 32-record rings, 256 threads -- ~8 records per bucket per sub-step
      // -- so two workgroups share a CU)
      J.T = P.kn.narrow_unit == 16 ? 256 : 512;
      const int nr = 8, ntl = 16;
      if (nr < J.R) {
        J.R = nr;
        for (JitCol& C : J.cols) C.frac = C.decode && (nr * C.bits) % 32 != 0;
      }
      J.TL = std::max(J.R, ntl);
    }
    for (int l = 0; l < nleaves; ++l) {
      J.leaf_col.push_back(K.leaf_col[l]);
      const int ri = P.roar_index[members[0]][l];
      if (P.rprog_on && P.leaf_phys[l] == PH_BITMAP) J.leaf_mode.push_back(LEAF_NONE);  // read via its program
      else if (P.mv_index[members[0]][l] >= 0) J.leaf_mode.push_back(LEAF_DOCMASK);  // pgx_mv_leaf_mask's doc mask
      else J.leaf_mode.push_back(ri >= 0 ? (P.roar[ri].neg ? LEAF_DOCMASK_NOT : LEAF_DOCMASK) : S0.leaf[l].mode);
    }
    if (P.rprog_on)
      for (size_t k = 0; k < P.dm_progs.size(); ++k) {
        J.leaf_col.push_back(-1);
        J.leaf_mode.push_back(P.rchunk ? LEAF_RCHUNK : LEAF_DOCMASK);
      }
    const ExecPlan::StarPlan& SP = P.star[members[0]];
    if (SP.on) {
      for (size_t k = 0; k < SP.ranges.size(); ++k) {
        J.leaf_col.push_back(-1);
        J.leaf_mode.push_back(LEAF_RANGES);
      }
      J.prog_op = SP.op;
      J.prog_arg = SP.arg;
    } else {
      for (int i = 0; i < K.prog_len; ++i) {
        J.prog_op.push_back(K.prog_op[i]);
        J.prog_arg.push_back(K.prog_arg[i]);
      }
    }
    for (int a = 0; a < K.num_aggs; ++a) {
      J.agg_kind.push_back(K.agg_kind[a]);
      J.agg_col.push_back(K.agg_col[a]);
    }
    for (int p = 0; p < K.num_planes; ++p) J.plane_op.push_back(K.plane_op[p]);
    J.num_planes = K.num_planes;
    J.group_mode = P.use_part ? int(G_EMIT) : int(K.group_mode);
    for (int g = 0; g < K.num_gcols; ++g) {
      J.gcol.push_back(K.gcol[g]);
      J.gmul.push_back(K.gmul[g]);
      J.gshift.push_back(K.gshift[g]);
      J.ghi.push_back(K.ghi[g] ? 1 : 0);
    }
    J.hash_slots = (J.group_mode == G_HASH64 || J.group_mode == G_HASH128) ? hash_slots : 0;
    if (P.use_part) {
      J.keybits = P.part_keybits;
      J.emit_col = P.part_vcol;
      J.part_bits = P.part_narrow ? kNarrow1Bits : 0;
      J.emit_dictid = P.part_dictid;
      J.part_slab = P.part_slab;
      J.part_narrow = P.part_narrow;
      J.narrow_vbits = P.part_narrow ? P.narrow_vd : 0;
      J.narrow_unit = P.kn.narrow_unit;
      J.prefetch2 = P.part_narrow && P.kn.prefetch2;
    }
    J.dense_slots = P.dense_slots;
    // COUNT + one integer SUM / AVG over a dense LDS table: one packed 64-bit add per row when, for every segment of
    // the group, its rows fit the count field and rows x value range fit the offset field (flushed per segment)
    if ((K.group_mode == G_DENSE_LDS || K.group_mode == G_HASH64 || K.group_mode == G_HASH128) &&
        K.num_planes == 2 && K.num_aggs == 1 && (K.agg_kind[0] == A_SUM || K.agg_kind[0] == A_AVG) && !P.use_part) {
      const int c = K.agg_col[0];
      if (c >= 0 && J.cols[c].img != IMG_NONE && !J.cols[c].fp) {
        int64_t maxdocs = 1, ntiles = 0;
        uint64_t vrange = 0;
        const int64_t trows = int64_t(J.T) * J.TL;
        for (int sg : members) {
          maxdocs = std::max<int64_t>(maxdocs, P.ksegs[sg].num_docs);
          vrange = std::max<uint64_t>(vrange, P.segcols[sg][c]->vrange);
          ntiles += (int64_t(P.ksegs[sg].num_docs) + trows - 1) / trows;
        }
        // a workgroup flushes its table at every segment switch and walks at most ceil(tiles / CUs) tiles (the
        // persistent grid has at least one workgroup per CU): the rows one flush covers are bounded by both
        maxdocs = std::min<int64_t>(maxdocs, (ntiles + cus - 1) / cus * trows);
        const int cb = bits_for(maxdocs + 1);
        const long double sum_max = (long double)maxdocs * (long double)(vrange + 1);
        int sb = 0;
        while (sb < 64 && std::ldexp(1.0L, sb) <= sum_max) ++sb;
        if (cb + sb <= 64) J.dense_pack = 64 - cb;
      }
    }
    if (hp1 && !J.dense_pack && hashg) {  // the packed add does not fit after all: two planes per slot
      hp1 = false;
      while (hash_slots > 512 && lds_need() > lds_budget) hash_slots /= 2;
      J.hash_slots = hash_slots;
    }
    J.leafmask = P.fsm_on && P.lmask_off[members[0]] >= 0;
    J.compact = P.rchunk && !P.use_part;  // selective bitmap filters: aggregate the selected rows packed
    J.selmask = P.want_selmask;

    ExecPlan::JitGroup G;
    G.T = J.T;
    int lds_bytes = 0;
    std::string err;
    G.fn = jit_function(J, ctx->device, &lds_bytes, &err);
    if (!G.fn) fail(PGX_ERR_INTERNAL, "query kernel compile: " + err);
    // per-segment arguments
    const int64_t tile_rows = int64_t(J.T) * J.TL;
    int64_t tiles = 0;
    for (int s : members) {
      const KSeg& S = P.ksegs[s];
      JSeg js{};
      js.tile_begin = tiles;
      js.num_docs = S.num_docs;
      js.rec_base = P.rec_base[s];
      js.lmask = S.lmask;
      js.lmask_words = S.lmask_words;
      js.selmask = P.want_selmask ? P.sel_buf.as<unsigned int>() + P.sel_off[s] : nullptr;
      if (P.star[s].on) {
        // visit only the tiles that intersect a star-tree range: every selected doc lies in one
        auto& tl = P.star_tiles[s];
        tl.clear();
        for (const auto& r : P.star[s].ranges)
          for (int k = 0; k < r.second; ++k) {
            const int32_t a = P.blob32[r.first + 2 * k], b = P.blob32[r.first + 2 * k + 1];
            for (int64_t t = a / tile_rows; t <= b / tile_rows; ++t)
              if (tl.empty() || tl.back() != int32_t(t)) tl.push_back(int32_t(t));
          }
        std::sort(tl.begin(), tl.end());
        tl.erase(std::unique(tl.begin(), tl.end()), tl.end());
        const size_t off = star_tile_off;
        star_tile_off += tl.size();
        if (star_tile_off > P.star_tile_cap) fail(PGX_ERR_INTERNAL, "star tile list overflow");
        std::memcpy(B.host.bytes() + B.off_tiles + off * 4, tl.data(), tl.size() * 4);
        js.tiles = reinterpret_cast<const int*>(B.dev() + B.off_tiles + off * 4);
        tiles += int64_t(tl.size());
      } else {
        tiles += (int64_t(S.num_docs) + tile_rows - 1) / tile_rows;
      }
      for (int c = 0; c < nc; ++c) {
        const StagedColumn& col = *P.segcols[s][c];
        js.fwd[c] = S.fwd[c];
        js.dict[c] = S.dict[c];
        js.remap[c] = S.remap[c];
        js.img[c] = J.cols[c].img != IMG_NONE ? col.img_dev : nullptr;
        js.img_words[c] = J.cols[c].img != IMG_NONE ? col.img_words : 0;
        js.vbase[c] = col.vbase;
      }
      js.emit_rebase = !(P.use_part && P.part_vcol >= 0) ? 0
                       : (P.part_fp || (P.part_narrow && P.narrow_img == 5))
                           ? P.part_fbase[size_t(s)]  // the segment's dictionary in the concatenation / value table
                                   : P.segcols[s][P.part_vcol]->vbase - P.part_vbase;
      if (P.rprog_on)
        for (size_t k = 0; k < P.dm_progs.size(); ++k)
          js.lbits[nleaves + k] = P.rchunk ? reinterpret_cast<const uint32_t*>(P.rprog_dev + s * P.dm_progs.size() + k)
                                           : P.masks_dev + uintptr_t(P.rprogs[size_t(s) * P.dm_progs.size() + k].mask);
      for (int l = 0; l < nleaves; ++l) {
        const KLeaf& L = S.leaf[l];
        const int ri = P.roar_index[s][l];
        js.lbits[l] = (ri >= 0 && !P.rprog_on) ? P.masks_dev + P.roar[ri].mask_off : L.bitset;
        js.lranges[l] = L.ranges;
        js.lnr[l] = L.nranges;
        js.llo[l] = uint32_t(L.lo);
        js.lspan[l] = uint32_t(L.hi) - uint32_t(L.lo);
      }
      if (P.star[s].on)
        for (size_t k = 0; k < P.star[s].ranges.size(); ++k) {
          js.lranges[nleaves + k] = reinterpret_cast<const int*>(B.dev()) + P.star[s].ranges[k].first;
          js.lnr[nleaves + k] = P.star[s].ranges[k].second;
        }
      G.segs.push_back(js);
    }
    const int waves = J.T / 64;
    int per_cu = std::max(1, 32 / waves);
    const int64_t lds_all = std::max<int64_t>(lds, lds_bytes);  // incl. record staging (G_EMIT)
    if (lds_all > 0) per_cu = std::min<int64_t>(per_cu, std::max<int64_t>(1, (160 * 1024) / (lds_all + 256)));
    per_cu = std::min(per_cu, jit_occupancy(G.fn, J.T));  // registers too: a persistent grid one round deep
    const int64_t max_grid = int64_t(cus) * per_cu;
    const int64_t tpw = std::max<int64_t>(1, (tiles + max_grid - 1) / max_grid);
    G.grid = int(std::max<int64_t>(1, (tiles + tpw - 1) / tpw));
    std::memcpy(B.host.bytes() + B.off_jsegs + jidx * sizeof(JSeg), G.segs.data(), G.segs.size() * sizeof(JSeg));
    G.args.segs = reinterpret_cast<const JSeg*>(B.dev() + B.off_jsegs + jidx * sizeof(JSeg));
    jidx += G.segs.size();
    G.args.num_segs = int(G.segs.size());
    G.args.rdesc = P.rdesc_dev;
    G.args.total_tiles = tiles;
    G.args.tiles_per_wg = tpw;
    if (P.part_slab && tiles > 0) {
      G.args.part_wg_base = P.part_nwg;
      P.part_nwg += G.grid;
      P.part_wg_rows = std::max<int64_t>(P.part_wg_rows, tpw * tile_rows);
    }
    if (tiles > 0) P.jit.push_back(std::move(G));
  }
  if (P.jit.empty()) P.jit.push_back(ExecPlan::JitGroup{});  // every segment empty: nothing to launch
}

void launch_fsm(ExecPlan& P, hipStream_t st) {
  if (!P.fsm_on) return;
  PGX_LAUNCH(st, "pgx_fsm", pgx_launch_fsm(P.fsm_segbuf.as<FsmSeg>(), int(P.fsm_segs.size()), P.fsm_table.as<uint32_t>(),
                           P.fsm.num_states, P.fsm.num_leaves, P.fsm_chunks, P.fsm_cnt.as<uint32_t>(),
                           P.fsm_stv.as<uint16_t>(), P.fsm_pcount.as<unsigned long long>(), P.fsm_pstate.as<uint16_t>(),
                           P.fsm_T, P.kq.stats, st),
            "statistics automaton launch");
}

void launch_scan(ExecPlan& P, hipStream_t st) {
  if (!P.mv_items.empty()) {
    if (P.jit.empty() || !P.jit[0].fn) fail(PGX_ERR_UNSUPPORTED, "multi-value filter needs the query kernels");
    PGX_LAUNCH(st, "pgx_mv_leaf_mask", pgx_launch_mv_leaf_mask(P.mv_descs.as<MvLeaf>(), int(P.mv_items.size()), P.mv_max_words, st),
              "multi-value leaf masks");
  }
  if (!P.jit.empty()) {
    // a lone query's replay: bitmap programs and query kernel in two halves of the segment list, the second half's
    // programs on the side stream, so they run beside the first half's query kernel instead of before it
    const bool two = P.split2 && P.rdesc_dev && P.rprog_on && !P.roar_early && !P.rchunk && P.jit.size() == 1 &&
                     P.jit[0].fn && !P.fsm_on && P.mv_items.empty() && P.jit[0].segs.size() >= 64 &&
                     P.jit[0].segs.size() == P.ksegs.size() && !P.dm_progs.empty() &&
                     P.rprogs.size() == P.ksegs.size() * P.dm_progs.size() && P.ctx_side && !P.use_part;
    if (two) {
      ExecPlan::JitGroup& G = P.jit[0];
      const int n = int(G.segs.size()), h = std::max(1, n / P.kn.lone_head);
      const int ph = h * int(P.dm_progs.size());
      hip_check(hipEventRecord(P.ev_pre.get(), st), "event");
      hip_check(hipStreamWaitEvent(P.ctx_side, P.ev_pre.get(), 0), "event wait");
      launch_bitmaps(P, st, 0, ph);
      launch_bitmaps(P, P.ctx_side, ph, int(P.rprogs.size()));
      hip_check(hipEventRecord(P.ev_half.get(), P.ctx_side), "event");
      const long long tiles = G.args.total_tiles, th = G.segs[h].tile_begin;
      for (int half = 0; half < 2; ++half) {
        if (half) hip_check(hipStreamWaitEvent(st, P.ev_half.get(), 0), "event wait");
        JArgs a = G.args;
        a.agg_out = P.kq.agg_out;
        a.stats = P.kq.stats;
        a.table = P.kq.table;
        a.hkeys = P.kq.keys;
        a.hstate = P.kq.key_state;
        a.hash_cap = P.kq.hash_cap;
        a.overflow = P.kq.overflow;
        a.segs = G.args.segs + (half ? h : 0);
        a.num_segs = half ? n - h : h;
        a.tile_base = half ? th : 0;
        a.total_tiles = half ? tiles : th;
        // the whole persistent grid for each half (the plan's tiles per workgroup were sized for all the tiles)
        const long long span = half ? tiles - th : th;
        const long long tph = std::max<long long>(1, (span + G.grid - 1) / G.grid);
        a.tiles_per_wg = tph;
        const int grid = int(std::max<long long>(1, (span + tph - 1) / tph));
        void* params[] = {&a};
        PGX_LAUNCH(st, "pgxq", hipModuleLaunchKernel(static_cast<hipFunction_t>(G.fn), grid, 1, 1, G.T, 1, 1, 0, st,
                                                     params, nullptr),
                   "query kernel launch");
      }
      return;
    }
    if (P.rdesc_dev && !P.roar_early) launch_bitmaps(P, st);
    P.roar_early = false;  // relaunches (hash-table retries, timed iterations) expand again
    for (auto& G : P.jit) {
      if (!G.fn) continue;
      G.args.agg_out = P.kq.agg_out;
      G.args.stats = P.kq.stats;
      G.args.table = P.kq.table;
      G.args.part_cursor = P.part_cursor;
      G.args.part_overflow = P.part_overflow;
      G.args.part_cap = P.part_cap;
      G.args.part_cstride = P.part_slab ? 1 : kCursorStride;
      G.args.part_nwg = P.part_nwg;
      G.args.part_hi = P.part_hi;
      G.args.hkeys = P.kq.keys;
      G.args.hstate = P.kq.key_state;
      G.args.hash_cap = P.kq.hash_cap;
      G.args.overflow = P.kq.overflow;
      void* params[] = {&G.args};
      PGX_LAUNCH(st, "pgxq", hipModuleLaunchKernel(static_cast<hipFunction_t>(G.fn), G.grid, 1, 1, G.T, 1, 1, 0, st, params,
                                      nullptr),
                "query kernel launch");
    }
    launch_fsm(P, st);
    return;
  }
  if (P.kq.total_tiles == 0) return;
  if (P.rprog_on) fail(PGX_ERR_INTERNAL, "bitmap programs need the query kernels");
  PGX_LAUNCH(st, "pgx_scan_kernel", pgx_launch_scan(&P.kq, P.grid, P.tiles_per_wg, P.lds_bytes, st), "scan kernel launch");
  launch_fsm(P, st);
}

void finish_result(pgx_ctx* ctx, const pgx_query& q, ExecPlan& P, ExecBuffers& B, pgx_segment* const* segs, int n,
                   hipStream_t st, pgx_result* R, const unsigned long long* dense_host_override) {
  KQuery& K = P.kq;
  unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
  const bool hash = hash_mode(K.group_mode);
  if (!dense_host_override && B.tbl_live && K.num_gcols > 0 && !hash) {
    // in-arena dense table: outputs and table in ONE read-back, occupied slots found on the host
    hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes + B.tbl_bytes, hipMemcpyDeviceToHost, st),
              "outputs + table D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    prof_mark("f.sync");
    dense_host_override = outs + kOutsBytes / 8;
  }
  const bool dense_dev = K.num_gcols > 0 && !hash && !dense_host_override;
  // group-by compaction (occupied slots -> columnar), read back together with the outputs block: ONE sync
  const uint64_t slots = hash ? P.hash_cap : P.dense_slots;
  std::vector<int64_t> slot_ids;
  std::vector<unsigned long long> planes;  // [plane][group]
  std::vector<unsigned long long> gkeys;  // hash keys of the groups: key_words words each
  uint64_t ng = 0;
  // first guess of the group count: the plan's previous execution's (a kept plan replays the same query), else <= 64k
  auto guess = [&](uint64_t limit) {
    const uint64_t g = P.last_groups ? std::max<uint64_t>(256, P.last_groups + P.last_groups / 4) : (uint64_t(1) << 16);
    return std::max<uint64_t>(1, std::min<uint64_t>(limit, g));
  };
  if (dense_dev) {
    // a table of the plan's own of up to 64K slots is read whole, so the compaction can put it back clean (below)
    const bool own = B.table.p && K.table == devp(B.table);
    uint64_t cap = own && slots <= 65536 ? slots : guess(slots);
    for (;;) {
      const size_t bytes = 256 + size_t(cap) * 8 * (1 + K.num_planes);
      DevBuf res(ctx, bytes);
      PinnedBuf hres(ctx, bytes);
      hip_check(hipMemsetAsync(res.p, 0, 8, st), "memset");
      unsigned long long* rb = devp(res);
      // the plan's own table, read whole: put its slots back to their initial values for the next execution
      const bool reset = own && cap >= slots && slots <= (uint64_t(1) << 20) && K.num_planes <= 32;
      uint32_t min_mask = 0;
      for (int p = 0; p < K.num_planes; ++p)
        if (K.plane_op[p] == P_MIN_ORD) min_mask |= 1u << p;
      PGX_LAUNCH(st, "pgx_compact", pgx_launch_compact(K.table, slots, K.num_planes, rb, reinterpret_cast<int64_t*>(rb + 32), rb + 32 + cap,
                                   cap, reset ? 1 : 0, min_mask, st),
                "compact");
      hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
      hip_check(hipMemcpyAsync(hres.p, res.p, bytes, hipMemcpyDeviceToHost, st), "groups D2H");
      hip_check(hipStreamSynchronize(st), "sync");
      prof_mark("f.sync");
      const unsigned long long* h = reinterpret_cast<const unsigned long long*>(hres.p);
      const uint64_t cnt = h[0];
      if (cnt > cap) {  // more groups than the guess: once more at the exact size
        cap = cnt;
        continue;
      }
      B.table_clean = reset;
      ng = cnt;
      slot_ids.assign(reinterpret_cast<const int64_t*>(h + 32), reinterpret_cast<const int64_t*>(h + 32) + ng);
      planes.resize(ng * K.num_planes);
      for (int p = 0; p < K.num_planes; ++p)
        std::memcpy(planes.data() + p * ng, h + 32 + cap + p * cap, ng * 8);
      break;
    }
    P.last_groups = ng;
  } else if (hash && K.num_gcols > 0) {
    // compaction, key gather and read-back of the live groups in ONE round trip at the guessed size (the gather reads
    // the group count on the device); again at the exact size if the guess was short
    // (the outputs block travels with the groups; at most one group per slot)
    const uint64_t cap_max = std::max<uint64_t>(1, slots);
    const uint64_t kw = uint64_t(K.key_words);
    uint64_t cap = guess(cap_max);
    for (;;) {
      const size_t bytes = 256 + size_t(cap) * 8 * (1 + K.num_planes + kw);
      DevBuf res(ctx, bytes);
      PinnedBuf hres(ctx, bytes);
      unsigned long long* rb = devp(res);
      int64_t* oslot = reinterpret_cast<int64_t*>(rb + 32);
      unsigned long long* oplanes = rb + 32 + cap;
      unsigned long long* okeys = rb + 32 + cap * (1 + K.num_planes);
      hip_check(hipMemsetAsync(rb, 0, 8, st), "memset");
      PGX_LAUNCH(st, "pgx_compact", pgx_launch_compact(K.table, slots, K.num_planes, rb, oslot, oplanes, cap, 0, 0u, st),
                 "compact");
      PGX_LAUNCH(st, "pgx_gather_keys", pgx_launch_gather_keys(K.keys, oslot, rb, int64_t(cap), int(kw), okeys, st),
                 "gather keys");
      hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
      hip_check(hipMemcpyAsync(hres.p, res.p, bytes, hipMemcpyDeviceToHost, st), "groups D2H");
      hip_check(hipStreamSynchronize(st), "sync");
      prof_mark("f.sync");
      const unsigned long long* h = reinterpret_cast<const unsigned long long*>(hres.p);
      const uint64_t cnt = std::min<uint64_t>(h[0], cap_max);
      if (cnt > cap) {
        cap = cnt;
        continue;
      }
      ng = cnt;
      slot_ids.assign(reinterpret_cast<const int64_t*>(h + 32), reinterpret_cast<const int64_t*>(h + 32) + ng);
      planes.resize(ng * K.num_planes);
      for (int p = 0; p < K.num_planes; ++p) std::memcpy(planes.data() + p * ng, h + 32 + cap + p * cap, ng * 8);
      const unsigned long long* gk = h + 32 + cap * (1 + K.num_planes);
      gkeys.assign(gk, gk + ng * kw);
      break;
    }
    P.last_groups = ng;
  } else if (!dense_host_override) {  // one read-back of every output plane and statistic
    hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "outputs D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    prof_mark("f.sync");
  }
  const unsigned long long* stats = outs + 16;
  R->stats[0] = int64_t(stats[0]);
  R->stats[1] = int64_t(stats[1]) + P.host_entries;
  R->stats[2] = int64_t(stats[0]) * P.n_proj;
  R->stats[3] = P.total_raw;
  R->num_aggs = K.num_aggs;
  R->agg_fn = q.agg_fn;
  R->top_n = q.top_n;
  R->group_by = K.num_gcols > 0;
  R->mode = P.mode_ref;
  if (!R->group_by) {
    const unsigned long long* acc = outs;
    R->agg_value.assign(K.num_aggs, 0.0);
    R->agg_count.assign(K.num_aggs, 0);
    for (int a = 0; a < K.num_aggs; ++a) {
      const int fn = K.agg_kind[a];
      if (fn == A_COUNT) {
        R->agg_count[a] = int64_t(acc[0]);
        R->agg_value[a] = double(int64_t(acc[0]));
      } else {
        R->agg_value[a] = decode_plane(K.plane_op[a + 1], K.agg_fp[a], acc[a + 1], fn);
        R->agg_count[a] = int64_t(acc[0]);
      }
    }
    return;
  }
  if (dense_host_override) {
    for (uint64_t s = 0; s < slots; ++s)
      if (dense_host_override[s]) slot_ids.push_back(int64_t(s));
    ng = slot_ids.size();
    planes.resize(ng * K.num_planes);
    for (int p = 0; p < K.num_planes; ++p)
      for (uint64_t i = 0; i < ng; ++i) planes[p * ng + i] = dense_host_override[p * slots + slot_ids[i]];
  }
  prof_mark("f.groups");
  // ARRAY_BASED iteration order is ascending raw key (DefaultGroupKeyGenerator.java:613-644): sort dense slots.
  std::vector<uint64_t> order(ng);
  std::iota(order.begin(), order.end(), 0);
  if (!hash && ng > 1) {
    if (slots <= 64 * ng + 65536) {  // slot ids are distinct and < slots: place them (one pass over the slot range)
      std::vector<int64_t> at(slots, -1);
      for (uint64_t i = 0; i < ng; ++i) at[uint64_t(slot_ids[i])] = int64_t(i);
      uint64_t k = 0;
      for (uint64_t s = 0; s < slots; ++s)
        if (at[s] >= 0) order[k++] = uint64_t(at[s]);
    } else {
      std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return slot_ids[a] < slot_ids[b]; });
    }
  }
  R->num_groups = int64_t(ng);
  R->key_seg.assign(K.num_gcols, std::vector<int32_t>(ng));
  R->key_id.assign(K.num_gcols, std::vector<int32_t>(ng));
  for (uint64_t oi = 0; oi < ng; ++oi) {
    const uint64_t i = order[oi];
    for (int g = 0; g < K.num_gcols; ++g) {
      int64_t gid;
      if (!hash) {
        const uint64_t sl = uint64_t(slot_ids[i]);
        if (K.num_gcols == 1) gid = int64_t(sl);  // one column: the slot is the id
        else if (slots <= 0xFFFFFFFFull) gid = int64_t((uint32_t(sl) / uint32_t(K.gmul[g])) % uint32_t(P.gdicts[g].card));
        else gid = int64_t((sl / K.gmul[g]) % uint64_t(P.gdicts[g].card));
      } else {
        const unsigned long long w = gkeys[i * uint64_t(K.key_words) + uint64_t(K.ghi[g])];
        gid = int64_t((w >> K.gshift[g]) & ((1ull << P.gbits[g]) - 1ull));
      }
      R->key_seg[g][oi] = P.gdicts[g].rep_seg[gid];
      R->key_id[g][oi] = P.gdicts[g].rep_id[gid];
    }
  }
  R->g_value.assign(K.num_aggs, std::vector<double>(ng));
  R->g_count.assign(K.num_aggs, std::vector<int64_t>(ng));
  for (int a = 0; a < K.num_aggs; ++a) {
    for (uint64_t oi = 0; oi < ng; ++oi) {
      const uint64_t i = order[oi];
      const int64_t cnt = int64_t(planes[i]);
      R->g_count[a][oi] = cnt;
      if (K.agg_kind[a] == A_COUNT) R->g_value[a][oi] = double(cnt);
      else R->g_value[a][oi] = decode_plane(K.plane_op[a + 1], K.agg_fp[a], planes[(a + 1) * ng + i], K.agg_kind[a]);
      const int cp = P.g_count_plane.empty() ? -1 : P.g_count_plane[a];
      if (cp == -2) R->g_count[a][oi] = int64_t(planes[(a + 1) * ng + i]);
      else if (cp >= 0) R->g_count[a][oi] = int64_t(planes[uint64_t(cp) * ng + i]);
    }
  }
  prof_mark("f.decode");
}

uint64_t initial_hash_cap(pgx_segment* const* segs, int n, const ExecPlan& P) {
  uint64_t docs = 0;
  for (int s = 0; s < n; ++s) docs += uint64_t(segs[s]->total_raw_docs);
  uint64_t prod = 1;
  bool big = false;
  for (const auto& g : P.gdicts) {
    if (prod > (uint64_t(1) << 40) / uint64_t(g.card)) big = true;
    else prod *= uint64_t(g.card);
  }
  uint64_t want = std::max<uint64_t>(1024, std::min<uint64_t>(big ? docs : std::min(prod, docs), uint64_t(1) << 25));
  uint64_t cap = 1;
  while (cap < want * 2) cap <<= 1;
  return cap;
}


}  // namespace pgxh

namespace pgxh {


// PGX_DEBUG=host_profile: per-phase host wall time of every pgx_execute on stderr (host overhead hunting).
struct HostProf {
  bool on = false;
  std::chrono::steady_clock::time_point t0, last;
  std::string line;
  explicit HostProf(bool enable) : on(enable) {  // PGX_DEBUG=host_profile
    if (on) t0 = last = std::chrono::steady_clock::now();
  }
  void mark(const char* what) {
    if (!on) return;
    const auto t = std::chrono::steady_clock::now();
    line += std::string(" ") + what + "=" + std::to_string(std::chrono::duration<double, std::micro>(t - last).count());
    last = t;
  }
  ~HostProf() {
    if (on)
      std::fprintf(stderr, "[pgx host us] total=%.1f%s\n",
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(),
                   line.c_str());
  }
};

// Long segment lists (C5: 4096 segments) are planned and launched in batches: every batch is planned on a planner
// thread of its own (plan_query, the pinned argument arena, the query-kernel arguments) while the calling thread sends
// and launches the batches in order, so the GPU starts after the first (small) batch is planned and host planning
// (~1 us per segment single-threaded) overlaps the GPU instead of pacing it.  Every batch decodes its group keys
// against global dictionaries built over the WHOLE list (Domain), accumulates into batch 0's dense table and writes
// its statistics / aggregation planes into batch 0's output block, so the combine stays on the device and the result
// is read back once.  Aggregation-only and dense group-by plans only (sparse / hash plans size their tables from the
// whole list); false before anything was launched when the plan does not qualify.
bool run_batched(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
                 const pgx_exec_opts* opts, pgx_result* R, hipStream_t st, uint32_t xflags, HostProf& hp) {
  int bs = (xflags & PGX_X_THROUGHPUT) ? 0 : 512;
  if (q.kn.batch_segs >= 0) bs = q.kn.batch_segs;
  if (bs <= 0 || n < 2 * bs || !q.kn.jit) return false;
  const size_t L = q.leaf_col.size();
  std::vector<GlobalDict> full;
  for (int g = 0; g < int(q.group_cols.size()); ++g) full.push_back(group_dict(q, segs, n, g));
  hp.mark("b.dicts");
  // Batch sizes double from a small first batch up to bs: every batch is planned concurrently from t = 0, and batch k
  // (twice batch k - 1) is ready by the time the GPU has run batches 0 .. k - 1 (~1 us of planning per segment on one
  // planner thread against ~1.5 us of GPU time per C5 segment).
  const int first = std::max(1, std::min(64, bs));
  std::vector<int> start{0};
  for (int size = first; start.back() < n; size = std::min(bs, 2 * size)) {
    const int left = n - start.back();
    start.push_back(start.back() + (left < size + size / 2 ? left : size));  // a short tail joins the last batch
  }
  const int nb = int(start.size()) - 1;
  struct Batch {
    std::unique_ptr<ExecPlan> P;
    std::unique_ptr<ExecBuffers> B;
    bool ready = false, eligible = true;
    std::exception_ptr err;
  };
  std::vector<Batch> bt(nb);
  std::mutex mu;
  std::condition_variable cv;
  int done = 0;
  const int dev = ctx->device;
  std::vector<std::string> prof(hp.on ? nb : 0);  // PGX_DEBUG=host_profile: each planner's phase marks
  // set when batch 0 turns out ineligible: the tasks not yet started return at once (the caller re-plans the list)
  std::atomic<bool> cancel{false};
  auto plan_one = [&, dev](int b) {
    Batch& x = bt[b];
    if (b > 0 && cancel.load(std::memory_order_relaxed)) {
      std::lock_guard<std::mutex> g(mu);
      x.eligible = false;
      x.ready = true;
      ++done;
      cv.notify_all();
      return;
    }
    HostProf bp(hp.on);
    if (bp.on) g_prof_mark = [&bp](const char* w) { bp.mark(w); };
    try {
      hip_check(hipSetDevice(dev), "hipSetDevice");  // device buffers and JIT modules belong to the context's device
      const int s0 = start[b], cnt = start[b + 1] - s0;
      Domain d;
      d.g = &full;
      d.index.resize(cnt);
      std::iota(d.index.begin(), d.index.end(), s0);
      x.P = std::make_unique<ExecPlan>();
      x.P->serial = true;
      plan_query(ctx, q, segs + s0, cnt, bindings ? bindings + size_t(s0) * L : nullptr, xflags, *x.P, &d);
      const int gm = x.P->kq.group_mode;
      x.eligible = !x.P->use_part && (gm == G_NONE || gm == G_DENSE_LDS || gm == G_DENSE_GLOBAL) && x.P->mv_items.empty();
      if (x.eligible) {
        x.B = std::make_unique<ExecBuffers>();
        bp.mark("t.plan");
        build_arena(ctx, *x.P, *x.B);
        bp.mark("t.arena");
        plan_jit(ctx, q, segs + s0, cnt, *x.P, *x.B);
        bp.mark("t.jit");
      }
    } catch (...) {
      x.err = std::current_exception();
    }
    if (bp.on) {
      prof[b] = bp.line;
      bp.on = false;
      g_prof_mark = nullptr;
    }
    std::lock_guard<std::mutex> g(mu);
    x.ready = true;
    ++done;
    cv.notify_all();
  };
  // the planner tasks reference this frame (plan_one and what it captures are declared above): every submitted task
  // finishes before run_batched returns or throws
  struct Drain {
    std::mutex& mu;
    std::condition_variable& cv;
    int& done;
    int submitted = 0;
    ~Drain() {
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return done == submitted; });
    }
  } drain{mu, cv, done};
  for (int b = 0; b < nb; ++b) {
    ++drain.submitted;
    ctx->plan_submit([&plan_one, b] { plan_one(b); });
  }
  // Two streams: each batch's argument arena and bitmap programs go on the side stream, and the query stream waits
  // for them with an event.  The copies' SDMA latency and the bitmap programs of batch k + 1 then run while batch k's
  // query kernel streams the forward indexes, instead of between the query kernels.  Declared after the buffers:
  // on any exit both streams drain before the buffers return to the pool.
  const bool two = true;
  hipStream_t ss = ctx->side;
  struct Events {
    hipStream_t a, b;
    std::vector<hipEvent_t> ev;
    hipEvent_t make() {
      hipEvent_t e = nullptr;
      hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
      ev.push_back(e);
      return e;
    }
    ~Events() {
      if (ev.empty()) return;
      (void)hipStreamSynchronize(a);
      (void)hipStreamSynchronize(b);
      for (auto e : ev) (void)hipEventDestroy(e);
    }
  } evs{st, ss, {}};
  if (two) {  // the side stream starts after the work already queued on the query stream (a caller's stream)
    hipEvent_t e = evs.make();
    hip_check(hipEventRecord(e, st), "record");
    hip_check(hipStreamWaitEvent(ss, e, 0), "wait");
  }
  int64_t host_entries = 0, total_raw = 0;
  for (int b = 0; b < nb; ++b) {
    {
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return bt[b].ready; });
    }
    hp.mark("b.wait");
    Batch& x = bt[b];
    if (x.err) std::rethrow_exception(x.err);
    if (!x.eligible) {
      if (b == 0) {  // nothing launched yet: the caller plans the whole list at once
        cancel.store(true, std::memory_order_relaxed);
        return false;
      }
      fail(PGX_ERR_INTERNAL, "batched plans disagree");
    }
    ExecPlan& P = *x.P;
    ExecBuffers& B = *x.B;
    send_arena(P, B, ss);
    if (b == 0) {
      alloc_outputs(ctx, P, B, opts ? opts->dense_out : nullptr, opts ? opts->dense_out_bytes : 0);
      reset_outputs(P, B, ss);
    } else {
      const ExecPlan& P0 = *bt[0].P;
      const KQuery& K0 = P0.kq;
      if (P.kq.group_mode != K0.group_mode || P.dense_slots != P0.dense_slots || P.kq.num_planes != K0.num_planes)
        fail(PGX_ERR_INTERNAL, "batched plans disagree");
      alloc_outputs(ctx, P, B, K0.table, P0.dense_slots * uint64_t(K0.num_planes) * 8);
      reset_outputs(P, B, ss, false);
      P.kq.agg_out = K0.agg_out;  // one output block for the whole query
      P.kq.stats = K0.stats;
      P.kq.overflow = K0.overflow;
    }
    if (two) {
      hipEvent_t e = evs.make();
      hip_check(hipEventRecord(e, ss), "record");
      hip_check(hipStreamWaitEvent(st, e, 0), "wait");
    }
    launch_scan(P, st);
    hp.mark("b.launch");
    host_entries += P.host_entries;
    total_raw += P.total_raw;
  }
  hp.mark("batches");
  for (int b = 0; b < int(prof.size()); ++b) std::fprintf(stderr, "[pgx plan %d]%s\n", b, prof[b].c_str());
  ExecPlan& P0 = *bt[0].P;
  P0.host_entries = host_entries;
  P0.total_raw = total_raw;
  if (opts && (opts->flags & PGX_X_KEEP_DENSE_ON_DEVICE)) {
    unsigned long long* outs = reinterpret_cast<unsigned long long*>(bt[0].B->host.bytes() + bt[0].B->off_outs);
    hip_check(hipMemcpyAsync(outs, bt[0].B->dev() + bt[0].B->off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    const unsigned long long* stats = outs + 16;
    R->stats[0] = int64_t(stats[0]);
    R->stats[1] = int64_t(stats[1]) + P0.host_entries;
    R->stats[2] = int64_t(stats[0]) * P0.n_proj;
    R->stats[3] = P0.total_raw;
    R->group_by = true;
    R->num_aggs = P0.kq.num_aggs;
    R->agg_fn = q.agg_fn;
    return true;
  }
  finish_result(ctx, q, P0, *bt[0].B, segs, n, st, R, nullptr);
  hp.mark("finish");
  return true;
}

// After the launches of a non-partitioned plan: with PGX_X_KEEP_DENSE_ON_DEVICE the caller's dense table stays on the
// device (statistics only); otherwise the result is read back (finish_result).
void complete_scan(pgx_ctx* ctx, const pgx_query& q, ExecPlan& P, ExecBuffers& B, pgx_segment* const* segs, int n,
                   const pgx_exec_opts* opts, hipStream_t st, pgx_result* R) {
  if (opts && (opts->flags & PGX_X_KEEP_DENSE_ON_DEVICE)) {
    unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
    hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    const unsigned long long* stats = outs + 16;
    R->stats[0] = int64_t(stats[0]);
    R->stats[1] = int64_t(stats[1]) + P.host_entries;
    R->stats[2] = int64_t(stats[0]) * P.n_proj;
    R->stats[3] = P.total_raw;
    R->group_by = true;
    R->num_aggs = P.kq.num_aggs;
    R->agg_fn = q.agg_fn;
    return;
  }
  finish_result(ctx, q, P, B, segs, n, st, R, nullptr);
}

void run_query(pgx_ctx* ctx, const pgx_query& q, pgx_segment* const* segs, int n, const pgx_leaf_binding* bindings,
               const pgx_exec_opts* opts, pgx_result* R, const Domain* dom) {
  HostProf hp(q.kn.host_profile);
  if (hp.on) g_prof_mark = [&hp](const char* w) { hp.mark(w); };
  struct Unmark { ~Unmark() { g_prof_mark = nullptr; } } unmark;
  hipStream_t st = (opts && opts->stream) ? reinterpret_cast<hipStream_t>(opts->stream) : ctx->stream;
  const uint32_t xflags = opts ? opts->flags : 0;
  // plan cache (single-device plans without a caller key domain; only plain plans are ever kept, so a hit is one)
  const bool cache = !dom && plan_cache_on() && n > 0;
  std::vector<uint64_t> uids;
  uint64_t pkey = 0;
  if (cache) {
    pkey = plan_key(ctx, q, segs, n, bindings, xflags);
    if (auto e = plan_cache_acquire(&q, segs, n, pkey)) {
      struct Rel {
        const std::shared_ptr<PlanEntry>& e;
        ~Rel() { plan_cache_release(e); }
      } rel{e};
      hp.mark("cached");
      ExecPlan& P = *e->P;
      ExecBuffers& B = *e->B;
      if (P.use_part) {  // partitioned: scan, splits and aggregation into the kept slabs / buckets and partitions
        PartBuffers PB;
        bool ok = false;
        if (e->NB && replay_narrow(ctx, P, B, *e->NB, st)) {
          PB.okey = std::move(e->NB->okey);
          PB.oplane = std::move(e->NB->oplane);
          PB.prange = std::move(e->NB->prange);
          PB.ocap = e->NB->ocap;
          ok = true;
        } else if (e->PB && replay_part(ctx, P, B, *e->PB, st)) {
          PB.okey = std::move(e->PB->okey);
          PB.oplane = std::move(e->PB->oplane);
          PB.ocap = e->PB->ocap;
          ok = true;
        }
        if (ok) {
          hp.mark("launch");
          part_result(ctx, q, P, B, PB, R);
          hp.mark("finish");
          return;
        }
        e->key = ~e->key;  // (cannot happen: same inputs, same fills) never matched again; plan afresh below
      }
      // the device arena (descriptors, bitmap-program descriptors, blob) is as the first execution sent it; the
      // bitmap programs run again from launch_scan
      alloc_outputs(ctx, P, B, opts ? opts->dense_out : nullptr, opts ? opts->dense_out_bytes : 0);
      reset_outputs(P, B, st, true, true);
      P.split2 = !(xflags & PGX_X_THROUGHPUT);
      P.ctx_side = ctx->side;
      launch_scan(P, st);
      P.split2 = false;
      hp.mark("launch");
      complete_scan(ctx, q, P, B, segs, n, opts, st, R);
      hp.mark("finish");
      return;
    }
  }
  bool mv_group = false;  // a multi-value group column: key expansion per doc
  for (const auto& g : q.group_cols)
    for (int s = 0; s < n && !mv_group; ++s) mv_group = segs[s]->col(g).is_mv;
  bool mv_fn = false;
  for (int fn : q.agg_fn) mv_fn = mv_fn || fn >= PGX_COUNTMV;
  if (mv_group || (mv_fn && !q.group_cols.empty())) {
    // across devices the keys come from the shared Domain and the partials merge by key on the host (run_multi,
    // merge_host_groups); a caller-owned dense table is not offered (pgx_query_dense_slots reports -1)
    if (opts && opts->dense_out) fail(PGX_ERR_UNSUPPORTED, "multi-value group-by into a caller's dense table");
    run_mv_group(ctx, q, segs, n, bindings, xflags, R, st, dom);
    return;
  }
  if (mv_fn) {  // aggregation-only: the partials combine per function (combine_partial), on any device count
    run_mv(ctx, q, segs, n, bindings, xflags, R, st);
    return;
  }
  if (cache) {
    uids.resize(size_t(n));
    for (int s = 0; s < n; ++s) uids[size_t(s)] = segs[s]->uid;
  }
  const bool again = cache && plan_cache_seen_before(&q, pkey, uids);
  if (!dom && !again && run_batched(ctx, q, segs, n, bindings, opts, R, st, xflags, hp)) return;
  auto Pp = std::make_unique<ExecPlan>();
  auto Bp = std::make_unique<ExecBuffers>();
  ExecPlan& P = *Pp;
  plan_query(ctx, q, segs, n, bindings, xflags, P, dom);
  hp.mark("plan");
  ExecBuffers& B = *Bp;
  upload_plan(ctx, P, B, st);
  hp.mark("upload");
  plan_jit(ctx, q, segs, n, P, B);
  hp.mark("jit");
  if (P.use_part && P.part_cols.size() > 1) {  // several value columns: one pipeline run per column, joined by key
    if (run_value_columns(ctx, q, segs, n, P, B, st, R)) {
      hp.mark("finish");
      return;
    }
    P.use_part = false;
    P.jit.clear();
  }
  if (P.use_part) {
    if (P.part_narrow) {
      NarrowBuffers NB;
      if (run_narrow(ctx, P, B, NB, st)) {
        PartBuffers PB;
        PB.okey = std::move(NB.okey);
        PB.oplane = std::move(NB.oplane);
        PB.prange = std::move(NB.prange);
        PB.ocap = NB.ocap;
        part_result(ctx, q, P, B, PB, R);
        hp.mark("finish");
        if (cache && plan_cacheable(P))
          plan_cache_insert(&q, ctx, segs, n, std::move(uids), pkey, std::move(Pp), std::move(Bp),
                            std::make_unique<NarrowBuffers>(std::move(NB)));
        return;
      }
      narrow_fallback(ctx, q, segs, n, P, B);
    }
    PartBuffers PB;
    if (run_partitioned(ctx, P, B, PB, st)) {
      part_result(ctx, q, P, B, PB, R);
      hp.mark("finish");
      if (cache && plan_cacheable(P)) {
        auto kept = std::make_unique<PartBuffers>(std::move(PB));
        plan_cache_insert(&q, ctx, segs, n, std::move(uids), pkey, std::move(Pp), std::move(Bp), nullptr, std::move(kept));
      }
      return;
    }
    P.use_part = false;  // groups too many or too skewed for the partitions: global hash table, generic kernel
    P.jit.clear();
  }
  const bool hash = hash_mode(P.kq.group_mode);
  uint64_t hash_est = 0;
  if (hash) {
    P.hash_cap = hash_est = initial_hash_cap(segs, n, P);
    // the generated kernels pre-aggregate in LDS and send the global table distinct keys only: start at 1M slots, not
    // at one slot per row of a wide key space -- a 64M-slot table costs more to clear and compact than the scan (C7:
    // 330 ms of host and device per query).  An overflow reruns at the row-count estimate at once (C3-sized group
    // counts: one short failed pass -- every lane stops probing at the first overflow -- then one full pass)
    if (!P.jit.empty())
      P.hash_cap = std::min<uint64_t>(P.hash_cap, std::max<uint64_t>(uint64_t(1) << 20, q.hash_cap_hint.load()));
  }
  for (int attempt = 0; attempt < 6; ++attempt) {
    alloc_outputs(ctx, P, B, opts ? opts->dense_out : nullptr, opts ? opts->dense_out_bytes : 0);
    reset_outputs(P, B, st);
    launch_scan(P, st);
    hp.mark("launch");
    if (!hash) break;
    unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
    hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "sync");
    if (outs[24] == 0) break;
    if (P.kn.narrow_log)  // (PGX_DEBUG=narrow_log: which path ran, and why)
      std::fprintf(stderr, "[pgx hash] overflow %llu at %llu slots (attempt %d)\n", outs[24],
                   (unsigned long long)P.hash_cap, attempt);
    P.hash_cap = std::max(P.hash_cap * 4, hash_est);  // table full: grow and rerun
    if (attempt == 5) fail(PGX_ERR_OOM, "group-by hash table overflow");
  }
  if (hash && P.hash_cap > q.hash_cap_hint.load()) q.hash_cap_hint.store(P.hash_cap);
  complete_scan(ctx, q, P, B, segs, n, opts, st, R);
  hp.mark("finish");
  if (cache && plan_cacheable(P)) plan_cache_insert(&q, ctx, segs, n, std::move(uids), pkey, std::move(Pp), std::move(Bp));
}

}  // namespace pgxh

void pgx_result::ready() const {
  if (!async) return;
  async->join();
  if (async->status != PGX_OK) fail(async->status, async->msg);
}

// =================================================================================================
// C ABI
// =================================================================================================
extern "C" {

const char* pgx_last_error(void) { return g_last_error.c_str(); }
int32_t pgx_abi_version(void) { return PGX_ABI_VERSION; }

pgx_status pgx_ctx_create(const pgx_ctx_opts* opts, pgx_ctx** out) {
  return guarded([&] {
    if (!out) fail(PGX_ERR_INVALID_ARG, "out is NULL");
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    const int dev = opts ? opts->device : 0;
    if (dev < 0 || dev >= ndev) fail(PGX_ERR_DEVICE, "no HIP device " + std::to_string(dev));
    hip_check(hipSetDevice(dev), "hipSetDevice");
    auto* c = new pgx_ctx();
    c->device = dev;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
      c->num_cus = prop.multiProcessorCount;
    hip_check(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
    hip_check(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking), "hipStreamCreate");
    *out = c;
  });
}

// A context outlives its staged segments: pgx_ctx_destroy with segments still staged only drops the caller's
// reference, and the last pgx_segment_release frees the device memory (a JVM finaliser may release a segment after
// the context was closed).
void ctx_unref(pgx_ctx* ctx) {
  if (ctx->refs.fetch_sub(1) != 1) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->side);
  for (auto& kv : ctx->free_blocks) (void)hipFree(kv.second);
  for (auto& kv : ctx->live) (void)hipFree(kv.first);
  for (auto& kv : ctx->pinned_free) (void)hipHostFree(kv.second);
  for (auto& kv : ctx->pinned_live) (void)hipHostFree(kv.first);
  (void)hipStreamDestroy(ctx->stream);
  (void)hipStreamDestroy(ctx->side);
  delete ctx;
}

pgx_status pgx_ctx_destroy(pgx_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return;
    plan_cache_purge(nullptr, ctx);  // cached plans hold context references
    ctx_unref(ctx);
  });
}

pgx_status pgx_segment_stage(pgx_ctx* ctx, const pgx_segment_desc* d, pgx_segment** out) {
  return guarded([&] {
    if (!ctx || !d || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (d->total_docs < 0 || d->total_raw_docs < 0 || d->total_raw_docs > d->total_docs)
      fail(PGX_ERR_INVALID_ARG, "bad doc counts");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    auto seg = std::make_unique<pgx_segment>();
    seg->ctx = ctx;
    seg->name = d->name ? d->name : "";
    seg->total_docs = d->total_docs;
    seg->total_raw_docs = d->total_raw_docs;
    seg->cols.resize(d->num_columns);
    for (int i = 0; i < d->num_columns; ++i) {
      stage_column(ctx, seg.get(), d->columns[i], d->mem == PGX_MEM_DEVICE, seg->cols[i]);
      seg->by_name[seg->cols[i].name] = i;
      seg->names.push_back(seg->cols[i].name);
    }
    for (int i = 0; i < d->num_star_skip_dims; ++i)
      if (d->star_skip_dims && d->star_skip_dims[i]) seg->st_skip.emplace_back(d->star_skip_dims[i]);
    if (d->star_tree && d->star_tree_len) {
      const uint8_t* p = static_cast<const uint8_t*>(d->star_tree);
      seg->star_tree.assign(p, p + d->star_tree_len);
      parse_star_tree(*seg);
    }
    ctx->refs.fetch_add(1);  // released by pgx_segment_release
    *out = seg.release();
  });
}

pgx_status pgx_segment_release(pgx_segment* seg) {
  return guarded([&] {
    if (!seg) return;
    pgx_ctx* ctx = seg->ctx;
    delete seg;
    g_segment_frees.fetch_add(1);
    if (ctx) ctx_unref(ctx);
  });
}

pgx_status pgx_segment_device_bytes(const pgx_segment* seg, uint64_t* out) {
  return guarded([&] {
    if (!seg || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    *out = seg->device_bytes;
  });
}

pgx_status pgx_query_compile(pgx_ctx* ctx, const pgx_query_desc* d, pgx_query** out) {
  return guarded([&] {
    if (!ctx || !d || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    auto q = std::make_unique<pgx_query>();
    for (int a = 0; a < d->num_aggs; ++a) {
      const int fn = d->aggs[a].fn;
      if (fn < PGX_COUNT || fn > PGX_AVGMV) fail(PGX_ERR_UNSUPPORTED, "aggregation function not on the GPU path");
      q->agg_fn.push_back(fn);
      const char* c = d->aggs[a].column;
      std::string col = (c && std::strcmp(c, "*") != 0) ? c : "";
      if (fn != PGX_COUNT && col.empty()) fail(PGX_ERR_INVALID_ARG, "aggregation without column");
      q->agg_col.push_back(fn == PGX_COUNT ? "" : col);
    }
    for (int g = 0; g < d->num_group_cols; ++g) q->group_cols.push_back(d->group_cols[g]);
    q->top_n = d->top_n;
    q->filter.assign(d->filter, d->filter + d->num_filter_nodes);
    for (int l = 0; l < d->num_leaves; ++l) {
      q->leaf_col.push_back(d->leaves[l].column);
      q->leaf_kind.push_back(d->leaves[l].kind);
    }
    q->flags = d->flags;
    q->kn = read_knobs();
    *out = q.release();
  });
}

pgx_status pgx_query_set_key_domain(pgx_query* q, int32_t group_col, int32_t type, int64_t num_values,
                                    const int64_t* ivals, const double* dvals, const char* const* svals) {
  return guarded([&] {
    if (!q) fail(PGX_ERR_INVALID_ARG, "NULL query");
    if (group_col < 0 || group_col >= int(q->group_cols.size())) fail(PGX_ERR_INVALID_ARG, "group column index");
    plan_cache_purge(q, nullptr);  // plans decode keys against the domain
    if (num_values < 0 || num_values > INT32_MAX) fail(PGX_ERR_INVALID_ARG, "key domain size");
    q->key_domain.resize(q->group_cols.size());
    KeyDomain D;
    D.type = type;
    if (num_values == 0) {  // clears the domain: the union of the executed segments' dictionaries again
      q->key_domain[group_col] = KeyDomain{};
      return;
    }
    if (type == PGX_INT || type == PGX_LONG) {
      if (!ivals) fail(PGX_ERR_INVALID_ARG, "NULL values");
      D.iv.assign(ivals, ivals + num_values);
      for (int64_t i = 1; i < num_values; ++i)
        if (!(D.iv[i - 1] < D.iv[i])) fail(PGX_ERR_INVALID_ARG, "key domain not sorted and distinct");
    } else if (type == PGX_FLOAT || type == PGX_DOUBLE) {
      if (!dvals) fail(PGX_ERR_INVALID_ARG, "NULL values");
      D.dv.assign(dvals, dvals + num_values);
      for (int64_t i = 1; i < num_values; ++i)
        if (!(D.dv[i - 1] < D.dv[i])) fail(PGX_ERR_INVALID_ARG, "key domain not sorted and distinct");
    } else if (type == PGX_STRING) {
      if (!svals) fail(PGX_ERR_INVALID_ARG, "NULL values");
      for (int64_t i = 0; i < num_values; ++i) D.sv.emplace_back(svals[i] ? svals[i] : "");
      for (int64_t i = 1; i < num_values; ++i)
        if (!(D.sv[i - 1] < D.sv[i])) fail(PGX_ERR_INVALID_ARG, "key domain not sorted and distinct");
    } else {
      fail(PGX_ERR_INVALID_ARG, "key domain type");
    }
    D.set = true;
    q->key_domain[group_col] = std::move(D);
  });
}

pgx_status pgx_query_release(pgx_query* q) {
  return guarded([&] {
    plan_cache_purge(q, nullptr);
    delete q;
  });
}

pgx_status pgx_execute(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                       const pgx_leaf_binding* bindings, const pgx_exec_opts* opts, pgx_result** out) {
  return guarded([&] {
    if (!ctx || !q || !segs || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (!q->leaf_col.empty() && !bindings) fail(PGX_ERR_INVALID_ARG, "filter leaves need bindings");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    auto R = std::make_unique<pgx_result>();
    run_query(ctx, *q, segs, n, bindings, opts, R.get());
    *out = R.release();
  });
}

pgx_status pgx_result_release(pgx_result* r) {
  return guarded([&] { delete r; });  // an async result joins its execution first (~AsyncState)
}

struct PtrCardHash {
  size_t operator()(const std::pair<const uint32_t*, int>& k) const {
    return std::hash<const void*>()(k.first) ^ (size_t(k.second) * 0x9E3779B97F4A7C15ull);
  }
};

pgx_status pgx_execute_async(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                             const pgx_leaf_binding* bindings, const pgx_exec_opts* opts, pgx_result** out) {
  return guarded([&] {
    if (!ctx || !q || !segs || !out || n < 0) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    const size_t L = q->leaf_col.size();
    if (L && !bindings) fail(PGX_ERR_INVALID_ARG, "filter leaves need bindings");
    auto R = std::make_unique<pgx_result>();
    R->async = std::make_unique<AsyncState>();
    AsyncState& A = *R->async;
    A.segs.assign(segs, segs + n);
    if (L) {
      A.binds.assign(bindings, bindings + size_t(n) * L);
      A.words.reserve(A.binds.size());
      // one copy per distinct bitset (segments sharing a dictionary share their bindings' words, pgx_bind_predicates)
      std::unordered_map<std::pair<const uint32_t*, int>, const uint32_t*, PtrCardHash> copied;
      for (size_t i = 0; i < A.binds.size(); ++i) {
        pgx_leaf_binding& b = A.binds[i];
        if (!b.words) continue;
        const int card = segs[i / L]->col(q->leaf_col[i % L]).card;
        auto it = copied.find({b.words, card});
        if (it == copied.end()) {
          A.words.emplace_back(b.words, b.words + (card + 31) / 32);
          it = copied.emplace(std::make_pair(b.words, card), A.words.back().data()).first;
        }
        b.words = it->second;
      }
    }
    if (opts) {
      A.opts = *opts;
      A.has_opts = true;
    }
    pgx_result* r = R.get();
    AsyncPool::get().submit([ctx, q, r] {
      AsyncState& S = *r->async;
      const pgx_status st = guarded([&] {
        hip_check(hipSetDevice(ctx->device), "hipSetDevice");
        run_query(ctx, *q, S.segs.data(), int(S.segs.size()), S.binds.empty() ? nullptr : S.binds.data(),
                  S.has_opts ? &S.opts : nullptr, r);
      });
      std::lock_guard<std::mutex> g(S.m);
      S.status = st;
      if (st != PGX_OK) S.msg = g_last_error;
      S.done = true;
      S.cv.notify_all();
    });
    *out = R.release();
  });
}

pgx_status pgx_result_wait(pgx_result* r, int64_t timeout_ms) {
  if (!r) {
    g_last_error = "NULL argument";
    return PGX_ERR_INVALID_ARG;
  }
  if (!r->async) return PGX_OK;
  AsyncState& A = *r->async;
  {
    std::unique_lock<std::mutex> g(A.m);
    if (timeout_ms < 0) {
      A.cv.wait(g, [&] { return A.done; });
    } else if (!A.cv.wait_for(g, std::chrono::milliseconds(timeout_ms), [&] { return A.done; })) {
      g_last_error = "query still running";
      return PGX_ERR_TIMEOUT;
    }
  }
  A.join();
  if (A.status != PGX_OK) g_last_error = A.msg;
  return A.status;
}

pgx_status pgx_execute_multi(pgx_ctx* const* ctxs, int32_t nctx, const pgx_query* q, pgx_segment* const* segs,
                             int32_t n, const pgx_leaf_binding* bindings, const pgx_exec_opts* opts, pgx_result** out) {
  return guarded([&] {
    if (!ctxs || nctx < 1 || !q || !segs || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    for (int k = 0; k < nctx; ++k)
      if (!ctxs[k]) fail(PGX_ERR_INVALID_ARG, "NULL context");
    if (!q->leaf_col.empty() && !bindings) fail(PGX_ERR_INVALID_ARG, "filter leaves need bindings");
    if (opts && (opts->stream || opts->dense_out || (opts->flags & PGX_X_KEEP_DENSE_ON_DEVICE)))
      fail(PGX_ERR_INVALID_ARG, "pgx_execute_multi takes flags only (each context runs on its own stream)");
    auto R = std::make_unique<pgx_result>();
    run_multi(ctxs, nctx, *q, segs, n, bindings, opts ? opts->flags : 0, R.get());
    *out = R.release();
  });
}

pgx_status pgx_result_device_groups(const pgx_result* r, int64_t* n, void* records) {
  return guarded([&] {
    if (!r || !n) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    r->ready();
    if (!r->group_by || !r->lazy) fail(PGX_ERR_UNSUPPORTED, "the groups of this result are not in device memory");
    *n = r->num_groups;
    if (!records || !r->num_groups) return;
    const auto& L = *r->lazy;
    hip_check(hipSetDevice(L.ctx->device), "hipSetDevice");
    hipStream_t st = L.ctx->stream;
    PGX_LAUNCH(st, "pgx_group_pack", pgx_launch_group_pack(L.okey.as<uint64_t>(), L.oplane.as<uint64_t>(), L.ocap,
                                                           r->num_groups, L.nplanes, static_cast<uint64_t*>(records), st),
              "group pack");
    hip_check(hipStreamSynchronize(st), "sync");
  });
}

pgx_status pgx_result_record_words(const pgx_result* r, int32_t* words) {
  return guarded([&] {
    if (!r || !words) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    r->ready();
    if (!r->group_by || !r->lazy) fail(PGX_ERR_UNSUPPORTED, "the groups of this result are not in device memory");
    *words = 1 + r->lazy->nplanes;
  });
}

pgx_status pgx_result_merge_groups(pgx_ctx* ctx, const pgx_result* like, const void* records, int64_t n,
                                   const int64_t stats[4], pgx_result** out) {
  return guarded([&] {
    if (!ctx || !like || !out || n < 0 || (n && !records)) fail(PGX_ERR_INVALID_ARG, "bad argument");
    like->ready();
    if (!like->group_by || !like->lazy) fail(PGX_ERR_UNSUPPORTED, "template result has no device-resident groups");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    auto R = std::make_unique<pgx_result>();
    const uint64_t* rec = static_cast<const uint64_t*>(records);
    merge_device_groups(ctx, ctx->stream, rec, rec + 1, 1 + like->lazy->nplanes, 1, n, *like->lazy, R.get());
    R->num_aggs = like->num_aggs;
    R->agg_fn = like->agg_fn;
    R->top_n = like->top_n;
    R->mode = like->mode;
    for (int i = 0; i < 4; ++i) R->stats[i] = stats ? stats[i] : like->stats[i];
    *out = R.release();
  });
}

pgx_status pgx_result_stats(const pgx_result* r, int64_t out[4]) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    for (int i = 0; i < 4; ++i) out[i] = r->stats[i];
  });
}

pgx_status pgx_result_agg(const pgx_result* r, int32_t fn, double* value, int64_t* count) {
  return guarded([&] {
    if (r) r->ready();
    if (!r) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (r->group_by) fail(PGX_ERR_INVALID_ARG, "group-by result");
    if (fn < 0 || fn >= r->num_aggs) fail(PGX_ERR_INVALID_ARG, "function index");
    if (value) *value = r->agg_value[fn];
    if (count) *count = r->agg_count[fn];
  });
}

pgx_status pgx_result_num_groups(const pgx_result* r, int64_t* n) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !n) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    *n = r->num_groups;
  });
}

pgx_status pgx_result_group_keys(const pgx_result* r, int32_t c, int32_t* seg_index, int32_t* dict_id) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !r->group_by) fail(PGX_ERR_INVALID_ARG, "not a group-by result");
    const_cast<pgx_result*>(r)->materialize();
    if (c < 0 || c >= int(r->key_seg.size())) fail(PGX_ERR_INVALID_ARG, "group column index");
    if (seg_index) std::memcpy(seg_index, r->key_seg[c].data(), r->num_groups * 4);
    if (dict_id) std::memcpy(dict_id, r->key_id[c].data(), r->num_groups * 4);
  });
}

pgx_status pgx_result_group_values(const pgx_result* r, int32_t fn, double* value, int64_t* count) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !r->group_by) fail(PGX_ERR_INVALID_ARG, "not a group-by result");
    if (fn < 0 || fn >= r->num_aggs) fail(PGX_ERR_INVALID_ARG, "function index");
    const_cast<pgx_result*>(r)->materialize();
    if (value) std::memcpy(value, r->g_value[fn].data(), r->num_groups * 8);
    if (count) std::memcpy(count, r->g_count[fn].data(), r->num_groups * 8);
  });
}

pgx_status pgx_result_group_mode(const pgx_result* r, int32_t* mode) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !mode) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    *mode = r->mode;
  });
}

pgx_status pgx_result_trim(const pgx_result* r, int32_t fn, int64_t* idx, int64_t* n) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !r->group_by || !n) fail(PGX_ERR_INVALID_ARG, "not a group-by result");
    if (fn < 0 || fn >= r->num_aggs) fail(PGX_ERR_INVALID_ARG, "function index");
    const int64_t min_trim = std::max<int64_t>(r->top_n, 1000);
    const int64_t threshold = min_trim * 20, size = min_trim * 5;
    std::vector<int64_t> order;
    const std::vector<int64_t>* sel = &order;
    if (r->lazy && r->num_groups > threshold) {
      sel = &const_cast<pgx_result*>(r)->device_trim(fn, size);  // groups stay on the device
    } else if (r->num_groups <= threshold) {
      order.resize(r->num_groups);
      std::iota(order.begin(), order.end(), 0);
    } else {
      const int f = r->agg_fn[fn];
      const auto& v = r->g_value[fn];
      const auto& c = r->g_count[fn];
      auto key = [&](int64_t i) -> double {
        if (f == PGX_AVG || f == PGX_AVGMV) return c[i] ? v[i] / double(c[i]) : 0.0;  // AvgPair compares by ratio
        return v[i];
      };
      const bool asc = f == PGX_MIN || f == PGX_MINMV;
      auto cmp = [&](int64_t a, int64_t b) { return asc ? key(a) < key(b) : key(a) > key(b); };
      order.resize(r->num_groups);
      std::iota(order.begin(), order.end(), 0);
      std::nth_element(order.begin(), order.begin() + size, order.end(), cmp);
      order.resize(size);
      std::sort(order.begin(), order.end(), cmp);
    }
    if (idx) {
      if (*n < int64_t(sel->size())) fail(PGX_ERR_INVALID_ARG, "trim output capacity too small");
      std::memcpy(idx, sel->data(), sel->size() * 8);
    }
    *n = int64_t(sel->size());
  });
}

pgx_status pgx_result_gather(const pgx_result* r, const int64_t* gi, int64_t n, int32_t* seg_index, int32_t* dict_id,
                             double* value, int64_t* count) {
  return guarded([&] {
    if (r) r->ready();
    if (!r || !r->group_by || (n > 0 && !gi) || n < 0) fail(PGX_ERR_INVALID_ARG, "bad argument");
    for (int64_t j = 0; j < n; ++j)
      if (gi[j] < 0 || gi[j] >= r->num_groups) fail(PGX_ERR_INVALID_ARG, "group index out of range");
    if (n == 0) return;
    if (r->lazy) {
      const auto& L = *r->lazy;
      hip_check(hipSetDevice(L.ctx->device), "hipSetDevice");
      hipStream_t st = L.ctx->stream;
      DevBuf di(L.ctx, size_t(n) * 8), out(L.ctx, size_t(n) * (1 + L.nplanes) * 8);
      std::vector<uint64_t> h(size_t(n) * (1 + L.nplanes));
      hip_check(hipMemcpyAsync(di.p, gi, size_t(n) * 8, hipMemcpyHostToDevice, st), "gather H2D");
      PGX_LAUNCH(st, "pgx_group_gather", pgx_launch_group_gather(L.okey.as<uint64_t>(), L.oplane.as<uint64_t>(), L.ocap, L.nplanes,
                                        di.as<int64_t>(), n, out.as<uint64_t>(), st),
                "gather launch");
      hip_check(hipMemcpyAsync(h.data(), out.p, h.size() * 8, hipMemcpyDeviceToHost, st), "gather D2H");
      hip_check(hipStreamSynchronize(st), "sync");
      r->decode_lazy(h.data(), h.data() + n, n, n, seg_index, dict_id, value, count);
      return;
    }
    for (size_t c = 0; c < r->key_seg.size(); ++c)
      for (int64_t j = 0; j < n; ++j) {
        if (seg_index) seg_index[c * n + j] = r->key_seg[c][gi[j]];
        if (dict_id) dict_id[c * n + j] = r->key_id[c][gi[j]];
      }
    for (int a = 0; a < r->num_aggs; ++a)
      for (int64_t j = 0; j < n; ++j) {
        if (value) value[a * n + j] = r->g_value[a][gi[j]];
        if (count) count[a * n + j] = r->g_count[a][gi[j]];
      }
  });
}

pgx_status pgx_query_dense_slots(const pgx_query* q, pgx_segment* const* segs, int32_t n, int64_t* slots) {
  return guarded([&] {
    if (!q || !segs || !slots) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (!q->group_cols.empty() && query_is_mv(*q, segs, n)) {  // multi-value group-by: merged by key, never densely
      *slots = -1;
      return;
    }
    uint64_t prod = 1;
    for (int g = 0; g < int(q->group_cols.size()); ++g) prod *= uint64_t(group_dict(*q, segs, n, g).card);
    *slots = int64_t(prod);
  });
}

pgx_status pgx_query_dense_plane_op(const pgx_query* q, pgx_segment* const* segs, int32_t n, int32_t plane,
                                    int32_t* op) {
  return guarded([&] {
    if (!q || !segs || !op) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    if (plane == 0) { *op = P_ADD_I64; return; }
    if (plane < 1 || plane > int(q->agg_fn.size())) fail(PGX_ERR_INVALID_ARG, "plane");
    const int fn = q->agg_fn[plane - 1];
    if (fn == PGX_COUNT) { *op = P_ADD_I64; return; }
    const StagedColumn& c = segs[0]->col(q->agg_col[plane - 1]);
    const bool fp = c.data_type == PGX_FLOAT || c.data_type == PGX_DOUBLE;
    *op = (fn == PGX_MIN) ? P_MIN_ORD : (fn == PGX_MAX) ? P_MAX_ORD : (fp ? P_ADD_F64 : P_ADD_I64);
  });
}

pgx_status pgx_result_from_dense(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                                 const void* dense_device, const int64_t stats[4], pgx_result** out) {
  return guarded([&] {
    if (!ctx || !q || !segs || !dense_device || !out) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    ExecPlan P;
    std::vector<pgx_leaf_binding> none(size_t(n) * q->leaf_col.size(), pgx_leaf_binding{0, -1, nullptr});
    plan_query(ctx, *q, segs, n, none.data(), 0, P);
    if (!(P.kq.group_mode == G_DENSE_LDS || P.kq.group_mode == G_DENSE_GLOBAL))
      fail(PGX_ERR_INVALID_ARG, "query is not dense");
    const uint64_t total = P.dense_slots * P.kq.num_planes;
    std::vector<unsigned long long> host(total);
    hip_check(hipMemcpy(host.data(), dense_device, total * 8, hipMemcpyDeviceToHost), "dense D2H");
    auto R = std::make_unique<pgx_result>();
    ExecBuffers B;
    B.host = PinnedBuf(ctx, kOutsBytes);
    B.off_outs = 0;
    std::memset(B.host.p, 0, kOutsBytes);
    reinterpret_cast<unsigned long long*>(B.host.p)[16] = static_cast<unsigned long long>(stats[0]);
    P.host_entries = stats[1];
    finish_result(ctx, *q, P, B, segs, n, ctx->stream, R.get(), host.data());
    R->stats[0] = stats[0];
    R->stats[1] = stats[1];
    R->stats[2] = stats[2];
    R->stats[3] = stats[3];
    *out = R.release();
  });
}

pgx_status pgx_bind_predicates(const pgx_query* q, pgx_segment* const* segs, int32_t n, const pgx_predicate* preds,
                               pgx_bindings** out) {
  return guarded([&] {
    if (!q || (!segs && n) || (!preds && !q->leaf_col.empty()) || !out || n < 0) fail(PGX_ERR_INVALID_ARG, "NULL argument");
    auto B = std::make_unique<pgx_bindings>();
    const size_t L = q->leaf_col.size();
    B->arr.assign(size_t(n) * L, pgx_leaf_binding{0, -1, nullptr});
    // one resolution per (leaf, distinct dictionary) and chunk of segments; consecutive segments usually share a
    // dictionary, so each leaf first compares with the previous segment's column before the map lookup.  Long segment
    // lists (C5: 4096) resolve their chunks in parallel on the context's pool; bitsets are owned per chunk (moving a
    // vector keeps its buffer, so the binding pointers stay valid when the chunks' bitsets are gathered).
    constexpr int kChunk = 256;
    const int nchunk = (n + kChunk - 1) / kChunk;
    std::vector<std::vector<std::vector<uint32_t>>> owned(nchunk);
    std::vector<std::exception_ptr> errs(nchunk);
    auto bind_chunk = [&](int ci) {
      try {
        using Key = std::tuple<size_t, uint64_t, int, int, int>;
        std::map<Key, size_t> memo;
        std::vector<const StagedColumn*> prev(L, nullptr);
        std::vector<size_t> prev_at(L, 0);
        for (int s = ci * kChunk; s < std::min(n, (ci + 1) * kChunk); ++s)
          for (size_t l = 0; l < L; ++l) {
            const StagedColumn& c = segs[s]->col(q->leaf_col[l]);
            pgx_leaf_binding& b = B->arr[size_t(s) * L + l];
            const StagedColumn* p = prev[l];
            if (p && p->dict_hash == c.dict_hash && p->card == c.card && p->data_type == c.data_type &&
                p->pad_char == c.pad_char) {
              b = B->arr[prev_at[l]];
              continue;
            }
            prev[l] = &c;
            prev_at[l] = size_t(s) * L + l;
            const Key key = std::make_tuple(l, c.dict_hash, c.card, c.data_type, c.pad_char);
            auto it = memo.find(key);
            if (it != memo.end()) {
              b = B->arr[it->second];
              continue;
            }
            std::vector<uint32_t> w;
            resolve_binding(c, q->leaf_kind[l], preds[l], b.lo, b.hi, w);
            if (!w.empty()) {
              owned[ci].push_back(std::move(w));
              b.words = owned[ci].back().data();
            }
            memo.emplace(key, size_t(s) * L + l);
          }
      } catch (...) {
        errs[ci] = std::current_exception();
      }
    };
    if (nchunk > 1 && n >= 1024) segs[0]->ctx->parallel_for(nchunk, bind_chunk);
    else
      for (int ci = 0; ci < nchunk; ++ci) bind_chunk(ci);
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
    for (auto& o : owned)
      for (auto& w : o) B->words.push_back(std::move(w));
    *out = B.release();
  });
}

const pgx_leaf_binding* pgx_bindings_array(const pgx_bindings* b) { return b ? b->arr.data() : nullptr; }

pgx_status pgx_bindings_release(pgx_bindings* b) {
  delete b;
  return PGX_OK;
}

pgx_status pgx_timing_start(pgx_ctx* ctx) {
  return guarded([&] {
    if (!ctx) fail(PGX_ERR_INVALID_ARG, "bad argument");
    if (g_kt.on.load()) fail(PGX_ERR_INVALID_ARG, "a timing window is already open");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hip_check(hipDeviceSynchronize(), "sync");  // every later launch starts after the reference event
    std::lock_guard<std::mutex> g(g_kt.mu);
    for (auto& r : g_kt.recs) {
      g_kt.spare.push_back(r.a);
      g_kt.spare.push_back(r.b);
    }
    g_kt.recs.clear();
    if (!g_kt.ref) hip_check(hipEventCreate(&g_kt.ref), "event");
    hip_check(hipEventRecord(g_kt.ref, ctx->stream), "record");
    hip_check(hipEventSynchronize(g_kt.ref), "sync");
    g_kt.on = true;
  });
}

pgx_status pgx_timing_stop(pgx_ctx* ctx, double out[3], char* json, uint64_t json_cap) {
  return guarded([&] {
    if (!ctx || !g_kt.on.load()) fail(PGX_ERR_INVALID_ARG, "no timing window open");
    g_kt.on = false;
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hip_check(hipDeviceSynchronize(), "sync");
    std::lock_guard<std::mutex> g(g_kt.mu);
    std::vector<std::pair<double, double>> iv;
    std::map<std::string, std::pair<int, double>> per;
    for (const auto& r : g_kt.recs) {
      float a = 0, b = 0;
      hip_check(hipEventElapsedTime(&a, g_kt.ref, r.a), "elapsed");
      hip_check(hipEventElapsedTime(&b, g_kt.ref, r.b), "elapsed");
      iv.emplace_back(a, std::max(a, b));
      auto& x = per[r.name];
      ++x.first;
      x.second += std::max(0.0f, b - a);
    }
    std::sort(iv.begin(), iv.end());
    double busy = 0, sum = 0, cs = 0, ce = -1;
    for (const auto& x : iv) {
      sum += x.second - x.first;
      if (ce < 0 || x.first > ce) {
        if (ce >= 0) busy += ce - cs;
        cs = x.first;
        ce = x.second;
      } else {
        ce = std::max(ce, x.second);
      }
    }
    if (ce >= 0) busy += ce - cs;
    const double span = iv.empty() ? 0.0 : ce - iv.front().first;
    if (out) {
      out[0] = busy;
      out[1] = sum;
      out[2] = span;
    }
    if (json && json_cap) {
      std::string s = "{";
      char buf[160];
      std::snprintf(buf, sizeof buf, "\"busy_ms\": %.6f, \"sum_ms\": %.6f, \"span_ms\": %.6f, \"launches\": %zu, \"kernels\": {",
                    busy, sum, span, iv.size());
      s += buf;
      bool first = true;
      for (const auto& kv : per) {
        std::snprintf(buf, sizeof buf, "%s\"%s\": [%d, %.6f]", first ? "" : ", ", kv.first.c_str(), kv.second.first,
                      kv.second.second);
        s += buf;
        first = false;
      }
      s += "}}";
      if (s.size() + 1 > json_cap) fail(PGX_ERR_INVALID_ARG, "json buffer too small");
      std::memcpy(json, s.c_str(), s.size() + 1);
    }
  });
}

pgx_status pgx_execute_timed(pgx_ctx* ctx, const pgx_query* q, pgx_segment* const* segs, int32_t n,
                             const pgx_leaf_binding* bindings, int32_t iters, double* total_ms, double* kernel_ms,
                             pgx_result** out) {
  return guarded([&] {
    if (!ctx || !q || !segs || iters < 1) fail(PGX_ERR_INVALID_ARG, "bad argument");
    hip_check(hipSetDevice(ctx->device), "hipSetDevice");
    hipStream_t st = ctx->stream;
    ExecPlan P;
    plan_query(ctx, *q, segs, n, bindings, 0, P);
    ExecBuffers B;
    upload_plan(ctx, P, B, st);
    plan_jit(ctx, *q, segs, n, P, B);
    P.roar_early = false;  // every timed iteration includes the bitmap expansion
    PartBuffers PB;
    NarrowBuffers NB;
    bool narrow = false;
    if (P.use_part && P.part_cols.size() > 1) {  // (several value columns: timed through the global hash table)
      P.use_part = false;
      P.jit.clear();
    }
    if (P.use_part && P.part_narrow) {  // untimed: checks the narrow capacities
      narrow = run_narrow(ctx, P, B, NB, st);
      if (!narrow) narrow_fallback(ctx, *q, segs, n, P, B);
    }
    if (P.use_part && !narrow && !run_partitioned(ctx, P, B, PB, st)) {  // untimed: settles the partition sizes
      P.use_part = false;
      P.jit.clear();
    }
    const bool hash = hash_mode(P.kq.group_mode);
    if (hash && !P.use_part) P.hash_cap = initial_hash_cap(segs, n, P);
    if (!P.use_part) alloc_outputs(ctx, P, B, nullptr, 0);
    std::vector<hipEvent_t> ev(2 * iters);
    for (auto& e : ev) hip_check(hipEventCreate(&e), "event");
    hipEvent_t t0, t1;
    hip_check(hipEventCreate(&t0), "event");
    hip_check(hipEventCreate(&t1), "event");
    hip_check(hipEventRecord(t0, st), "record");
    for (int i = 0; i < iters; ++i) {
      reset_outputs(P, B, st);
      if (narrow) narrow_prepare(P, NB, st);
      else if (P.use_part) part_prepare(P, PB, st);
      hip_check(hipEventRecord(ev[2 * i], st), "record");
      launch_scan(P, st);
      if (narrow) narrow_enqueue(ctx, P, NB, st);
      else if (P.use_part) part_enqueue(P, PB, st);
      hip_check(hipEventRecord(ev[2 * i + 1], st), "record");
    }
    hip_check(hipEventRecord(t1, st), "record");
    hip_check(hipEventSynchronize(t1), "sync");
    float tot = 0, k = 0;
    hip_check(hipEventElapsedTime(&tot, t0, t1), "elapsed");
    for (int i = 0; i < iters; ++i) {
      float x = 0;
      hip_check(hipEventElapsedTime(&x, ev[2 * i], ev[2 * i + 1]), "elapsed");
      k += x;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    if (total_ms) *total_ms = tot;
    if (kernel_ms) *kernel_ms = k / iters;
    if (out) {
      auto R = std::make_unique<pgx_result>();
      if (P.use_part) {
        unsigned long long* outs = reinterpret_cast<unsigned long long*>(B.host.bytes() + B.off_outs);
        hip_check(hipMemcpyAsync(outs, B.dev() + B.off_outs, kOutsBytes, hipMemcpyDeviceToHost, st), "D2H");
        if (narrow) {
          hip_check(hipMemcpyAsync(outs + 28, NB.ctr.p, 32, hipMemcpyDeviceToHost, st), "D2H");
          PB.okey = std::move(NB.okey);
          PB.oplane = std::move(NB.oplane);
          PB.ocap = NB.ocap;
        } else {
          hip_check(hipMemcpyAsync(outs + 28, devp(PB.ctr) + PB.ctr_words() - 4, 32, hipMemcpyDeviceToHost, st), "D2H");
        }
        hip_check(hipStreamSynchronize(st), "sync");
        part_result(ctx, *q, P, B, PB, R.get());
      } else {
        finish_result(ctx, *q, P, B, segs, n, st, R.get(), nullptr);
      }
      *out = R.release();
    }
  });
}

}  // extern "C"
