"""A/B harness for the narrow aggregation kernel alone (pgx_narrow.hip pgx_narrow_aggregate): second-stage records of
C3's shape synthesised on the device, the kernel launched through libpgx's internal launcher, timed with HIP events.

C3 (BASELINE configs[2]) feeds the aggregation 2^18 partitions (256 first-level buckets x 2^10 second-level) of ~3,800
records over ~64 groups each: a record is the key's remaining 16 mix bits | the metric's 16-bit dictId << 16.

    python tools/narrow_agg_bench.py [--img 2|3|4] [--reps 10]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--parts", type=int, default=1 << 18)
    ap.add_argument("--per", type=int, default=3815)   # 1e9 rows / 2^18 partitions
    ap.add_argument("--groups", type=int, default=64)  # 16.7M groups / 2^18
    ap.add_argument("--min-max", type=int, default=1)
    ap.add_argument("--sum", type=int, default=1)
    args = ap.parse_args()
    from pinot_amd import native as N
    L = N.lib()
    dev = torch.device("cuda:0")
    P, per, G = args.parts, args.per, args.groups
    cap2 = (per + 64 + 3) // 4 * 4
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    rb2 = 16
    # per partition: G distinct 16-bit keys; each record one of them (uniform) and a uniform dictId
    keys = torch.randint(0, 1 << rb2, (P, G), device=dev, generator=g, dtype=torch.int64)
    pick = torch.randint(0, G, (P, cap2), device=dev, generator=g)
    did = torch.randint(0, 65536, (P, cap2), device=dev, generator=g, dtype=torch.int64)
    kk = torch.gather(keys, 1, pick)[:, :per]
    # expected: distinct (partition, key) groups; the sum of every record's value
    exp_groups = int(torch.unique((torch.arange(P, device=dev).unsqueeze(1) << rb2) | kk).numel())
    rec = (torch.gather(keys, 1, pick) | (did << rb2)).to(torch.int64) & 0xFFFFFFFF
    recs = rec.to(torch.int32).contiguous()
    used_did = did[:, :per].contiguous()
    del keys, pick, did, rec, kk
    cnt2 = torch.full((P,), per, dtype=torch.int32, device=dev)
    # FOR16 image: 64 block bases + u16 offsets of C3's metric dictionary (value = 16 i + jitter)
    card = 65536
    vals = np.arange(card, dtype=np.int64) * 16 + (np.arange(card) * 2654435761 % 16)
    sh = 10
    bases = vals[::1 << sh][:64].astype(np.uint32)
    offs = (vals - np.repeat(bases.astype(np.int64), 1 << sh)[:card]).astype(np.uint16)
    img = torch.from_numpy(np.concatenate([bases, offs.view(np.uint32)]).view(np.int32).copy()).to(dev)
    img_sh = sh
    if args.img == 4:  # packed frame of reference: the smallest image over the block shifts
        best = None
        for bsh in range(0, 17):
            nblk = (card + (1 << bsh) - 1) >> bsh
            lo = np.minimum.reduceat(vals, np.arange(0, card, 1 << bsh))
            hi = np.maximum.reduceat(vals, np.arange(0, card, 1 << bsh))
            b = max(1, int(hi.__sub__(lo).max()).bit_length())
            words = nblk + (card * b + 31) // 32 + 1
            if b <= 16 and (best is None or words < best[0]):
                best = (words, bsh, b, nblk, lo)
        words, bsh, b, nblk, lo = best
        off = (vals - np.repeat(lo, 1 << bsh)[:card]).astype(np.uint64)
        bits = np.zeros(words - nblk, dtype=np.uint64)
        pos = np.arange(card, dtype=np.uint64) * np.uint64(b)
        w, o = (pos >> np.uint64(5)).astype(np.int64), pos & np.uint64(31)
        lo_part = (off << o) & np.uint64(0xFFFFFFFF)
        hi_part = off >> (np.uint64(32) - o)
        np.bitwise_or.at(bits, w, lo_part)
        np.bitwise_or.at(bits, w + 1, np.where(o > 0, hi_part, 0).astype(np.uint64))
        packed = np.concatenate([lo.astype(np.uint32), bits.astype(np.uint32)])
        img = torch.from_numpy(packed.view(np.int32).copy()).to(dev)
        img_sh = bsh | (b << 5) | (nblk << 10)
        print("packed image: shift %d, %d-bit offsets, %d words" % (bsh, b, words))
    ocap = P * 192
    okey = torch.empty(ocap, dtype=torch.int64, device=dev)
    oplane = torch.empty(4 * ocap, dtype=torch.int64, device=dev)
    ctr = torch.zeros(4, dtype=torch.int64, device=dev)
    prange = torch.zeros(8, dtype=torch.int64, device=dev)
    vdict = torch.from_numpy(vals).to(dev)
    exp_sum = int(vdict[used_did].sum().item())
    del used_did
    cb = int(np.ceil(np.log2(cap2 + 2)))
    cshift = 64 - cb
    fn = L.pgx_launch_narrow_aggregate
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_void_p,
                   C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                   C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    grid = ncu * (4 if args.img == 3 else 1)
    L.pgx_narrow_scratch_words.restype = C.c_int64
    sw = L.pgx_narrow_scratch_words(P, args.img, grid)
    scratch = torch.empty(sw, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    mm = args.min_max

    def launch():
        ctr.zero_()
        rc = fn(recs.data_ptr(), cnt2.data_ptr(), cap2, P, rb2, 34, 0, args.img, img.data_ptr(), img.numel(), img_sh,
                vdict.data_ptr(), args.sum, mm, mm, cshift, okey.data_ptr(), oplane.data_ptr(), ocap, ctr.data_ptr(),
                prange.data_ptr(), grid, scratch.data_ptr(), sw, 0, C.c_void_p(st.cuda_stream))
        assert rc == 0, rc

    launch()
    torch.cuda.synchronize()
    ms = []
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        launch()
        b.record(st)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    groups = int(ctr[0].item())
    cnt_ok = int(oplane[:groups].sum().item()) == P * per
    sum_ok = int(oplane[ocap:ocap + groups].sum().item()) == exp_sum if args.sum else None
    print("check: groups %d (expected %d), counts %s, sums %s" % (groups, exp_groups, cnt_ok, sum_ok))
    gb = P * per * 4 / 1e9
    print("img=%d grid=%d parts=%d records=%.3e groups=%d lost=%d ms median=%.3f min=%.3f  (%.2f TB/s of records)"
          % (args.img, grid, P, P * per, groups, int(ctr[3].item()), np.median(ms), min(ms), gb / np.median(ms)))


if __name__ == "__main__":
    main()
