#!/usr/bin/env python3
"""Build and time compile-time tuning variants of the library on one GPU.

    python tools/variants.py build            # here (hipcc), into heatmap_amd/_lib/variants/
    python tools/variants.py run [names...]   # on the GPU box: one process per variant

Each run times hm_count over the same resident cloud (1e9 hotspot points,
zooms 0-18 by default) and prints one JSON line per variant.
"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
VDIR = os.path.join(REPO, "heatmap_amd", "_lib", "variants")

VARIANTS = {
    "base": [],
    "nows": ["HM_L1_WS=0"],                  # level 1 through k_l1_fast only (the shipped default)
    "wslate": ["HM_WS_PREFETCH_LATE=1"],     # k_l1_ws: next tile's loads after the count
    "spunfused": ["HM_SP_FUSED=0"],          # <= 32-key buckets through k_small_sort / scan / k_small_emit (round 5)
    "spres": ["HM_SPW_RESIDENT=1"],          # k_small_sort / k_small_emit on grids of their resident blocks
    "agpad4": ["HM_AG_PADW=4u"],             # k_aggregate histogram rows padded by 4 words (8 shipped)
    "agnostage": ["HM_AG_STAGE=0"],          # hm_reg_pyramid7: per-level cell stores (no LDS staging)
    "spp8": ["HM_SPP_WAVES=8"],              # k_small_pairs: 8-wave blocks
    "sprows16": ["HM_SPP_ROWS=16"],          # k_small_pairs: 16 rows a round (7 blocks per CU with staging)
    "spnostage": ["HM_SPP_STAGE=0"],         # k_small_pairs: per-level cell stores (no LDS staging)
    "ws": ["HM_L1_WS=1"],                    # k_l1_ws (12 compute + 4 writer waves)
    "ws8": ["HM_L1_WS=1", "HM_WS_C=512"],                  # k_l1_ws: 8 compute + 8 writer waves, 8192-point tiles
    "ws10": ["HM_L1_WS=1", "HM_WS_C=640"],                 # k_l1_ws: 10 compute + 6 writer waves, 10240-point tiles
    "ws12": ["HM_L1_WS=1", "HM_WS_C=768"],                 # k_l1_ws: 12 compute + 4 writer waves, 12288-point tiles
    "stamps6w8": ["HM_STAMPS=6", "HM_L1_WS=1", "HM_WS_C=512"],
    "stamps6w10": ["HM_STAMPS=6", "HM_L1_WS=1", "HM_WS_C=640"],
    "stamps7": ["HM_STAMPS=7"],              # k_small_pairs: per-round phase cycles (worker 0 and the allocator)
    "stamps": ["HM_STAMPS=1"],               # phase stamps for tools/stamps.py (k_partition)
    "stamps1": ["HM_STAMPS=2"],              # k_project_partition
    "stamps2": ["HM_STAMPS=3"],              # k_partition_fr
    "stamps4": ["HM_STAMPS=4"],              # k_l1_fast
    "stamps5": ["HM_STAMPS=5"],              # k_aggregate
    "stamps6": ["HM_STAMPS=6", "HM_L1_WS=1"],              # k_l1_ws: per-block phase cycles summed over its tiles
    "l1old": ["HM_L1_FAST=0"],               # level 1 through k_project_partition (round 3)
    "l1m3": ["HM_L1_MERGE_MIN=3"],
    "l1m12": ["HM_L1_MERGE_MIN=12"],
    "l1nomerge": ["HM_L1_MERGE_MIN=65"],
    "t4k512": ["HM_P1_PPT=8", "HM_L1_WAVES=6"],            # 4096-point tiles, 3 blocks of 8 waves per CU
    "t4k256": ["HM_P1_THREADS=256", "HM_L1_WAVES=3"],      # 4096-point tiles, 3 blocks of 4 waves per CU
    "m16": ["HM_L1_MERGE_MIN=16"],
    # tuning knobs (compile-time macros of the shipped sources)
    "noskew": ["HM_SKEW_CUR=0"],
    "p1_512x8": ["HM_P1_PPT=8"],
    "rs3": ["HM_RUN_SHARD_BITS=3"],
    "rs4": ["HM_RUN_SHARD_BITS=4"],
    "p1_256x16": ["HM_P1_THREADS=256"],
    "t512_8k": ["HM_PN_THREADS=512"],
    "su2": ["HM_SU=2"],
    "su8": ["HM_SU=8"],
    "k2old": ["HM_K2_FR=0"],                # level 2 through k_partition (run streaming)
    "p1_1024x8": ["HM_P1_THREADS=1024", "HM_P1_PPT=8"],
    "p1_1024x16": ["HM_P1_THREADS=1024"],
    "p1_1024x8w8": ["HM_P1_THREADS=1024", "HM_P1_PPT=8", "HM_P1_WAVES=8"],
    "mr2": ["HM_MERGE_ROUNDS=2"],
    "p1g8": ["HM_P1_GROUP=8"],
    "p1g16": ["HM_P1_GROUP=16"],
    "p1ilp2": ["HM_P1_ILP=2"],
    "frg8": ["HM_FR_GROUP=8"],
    "fr512_4k": ["HM_FR_THREADS=512", "HM_TN=4096"],
    "fr512": ["HM_FR_THREADS=512"],                 # k_partition_fr: 512-thread blocks, 16 keys a thread
    "ta64k": ["HM_TA=65536"],
    "ta128k": ["HM_TA=131072"],
    "lz3": ["HM_LEVEL_ZOOMS=3"],            # levels z5, z8, z11 (zmax 18)
    "split256": ["HM_SPW_SPLIT=256"],       # narrow small-bucket instantiation up to 256 keys
    "sp1024": ["HM_SP_MAX=1024"],           # buckets of 1025-2048 keys to k_aggregate
    "sp512": ["HM_SP_MAX=512"],             # buckets of 513-2048 keys to k_aggregate
    "sp256": ["HM_SP_MAX=256", "HM_SPW_SPLIT=256"],   # buckets of 257-2048 keys to k_aggregate
    "agslow": ["HM_AG_FAST=0"],             # k_aggregate with the lane-0 merge on every key
    "agm4": ["HM_MERGE_MIN=4"],
    "agm16": ["HM_MERGE_MIN=16"],
    "ta512k": ["HM_TA=524288"],
    "ta1m": ["HM_TA=1048576"],
    "hot1k": ["HM_MAX_HOT=1024"],
    "hot1kta1m": ["HM_MAX_HOT=1024", "HM_TA=1048576"],
    "os8": ["HM_OS_IT=8"],
    "tn16k": ["HM_TN=16384"],
    "os24": ["HM_OS_IT=24"],                # one-sweep radix tiles of 6144 keys
    "os32": ["HM_OS_IT=32"],                # one-sweep radix tiles of 8192 keys
    "l1n6": ["HM_L1_NARROW=1", "HM_L1_WAVES=6"],   # k_l1_fast with 4-B staging, 3 blocks per CU (spills)
    "nofuse": ["HM_CS_FUSE=0"],                      # packed grouped records: one zoom step per cascade launch
    "cs2it8": ["HM_CS2_IT=8"],                       # k_cascade2: 2048-item tiles
    "cs2it12": ["HM_CS2_IT=12"],
    "l1nt0": ["HM_L1_NT=0"],                        # K1's point loads without the non-temporal hint
    "l1early": ["HM_L1_LATE_DEST=0"],
    "sh8": ["HM_L1_SHARD_TILES=8"],                 # level-1 digits sharded above 8 tiles of points (default 64)
    "sh2": ["HM_L1_SHARD_TILES=2"],
    "lb1": ["HM_OS_LB=1"],                           # one-sweep look-back: one predecessor per round trip
    "lb8": ["HM_OS_LB=8"],
    "sh4": ["HM_L1_SHARD_TILES=4"],
    "sh16": ["HM_L1_SHARD_TILES=16"],                # K1: destinations before the staging (round 4)
    "xr16": ["HM_XR_PPT=16"],                        # route scatter: 4096-cell tiles (default 2048)
    "xr4": ["HM_XR_PPT=4"],
    "xrc8": ["HM_XRC_PPT=8"],                        # route count: 8 cells a thread in flight (default 16)
    "mg16": ["HM_MG_PPT=16"],                        # k_mb_gather: 4096-cell tiles (default 2048)
    "mg4": ["HM_MG_PPT=4"],
    "mgc32": ["HM_MG_CHUNK=32768"],                   # 32K-cell chunks a block (default 16K)
    "mbtc64": ["HM_MB2_TC32=0"],                    # k_mb_merge2: u64 table counts
    "mb2k": ["HM_MB2_TS=2048", "HM_MB2_T=256"],      # k_mb_merge2 tables / block size (default 4096 / 512)
    "mb8k": ["HM_MB2_TS=8192", "HM_MB2_T=1024"],
    "mb4k256": ["HM_MB2_TS=4096", "HM_MB2_T=256"],
    "mb4k1024": ["HM_MB2_TS=4096", "HM_MB2_T=1024"],
    "l1n4": ["HM_L1_NARROW=1", "HM_L1_WAVES=4"],   # 4-B staging at 2 blocks per CU               # 16K-key partition items (half the (item, child) pairs)                  # one-sweep radix tiles of 2048 keys (4 blocks per CU)
}

# Timing-only experiments: text patches applied to a copy of the sources (the
# shipped kernels carry no experiment toggles).  Results are wrong; every
# access stays in bounds.
PATCH_DEFINES = {}
PATCHES = {
    # k_partition / k_aggregate run bodies: no global key loads
    "noload": [("hm_kernels.hip", "                        x[u] = kv[L.bv[r] + (v - L.pre[r])];",
                "                        x[u] = make_uint4(v, v * 3u, v * 5u, v * 7u);")],
    # level 1: no region reservation atomics (every tile writes at its region base)
    "noatom1": [("hm_kernels.hip", "if (d < F && cnt[q]) gpos[q] = atomicAdd(&a.fill[slot[q]], cnt[q]);",
                 "if (d < F && cnt[q]) gpos[q] = 0;")],
}
# k_l1_fast (level 1, whole tiles): compute without the point loads, loads
# without the key stores, and no region reservation atomics
PATCHES["l1noload"] = [("hm_kernels.hip", """            la[k] = lat2[k * HM_P1_THREADS + tid];
            lo[k] = lon2[k * HM_P1_THREADS + tid];""", """            la[k] = make_double2(40.0 + 1e-7 * (double)(tid + 1024 * k), 40.0 + 1.3e-7 * (double)(tid + 1024 * k));
            lo[k] = make_double2(-122.0 + 1e-7 * (double)(tid + 1024 * k), -122.0 + 1.7e-7 * (double)(tid + 1024 * k));""")]
PATCHES["l1nostore"] = [
    ("hm_kernels.hip", "auto put_cold = [&](uint2 e) { *(OutT*)(outb + (uint64_t)e.y * sizeof(OutT)) = (OutT)e.x; };",
     "auto put_cold = [&](uint2 e) { if (e.x == 0xFFFFFFFFu && e.y == 0x1234567u) *(OutT*)outb = (OutT)e.x; };"),
    ("hm_kernels.hip", "        *(uint16_t*)(houtb + (uint64_t)e.y * 2u) = (uint16_t)hk;",
     "        if (hk == 0xFFFFFFFFu && e.y == 0x1234567u) *(uint16_t*)houtb = (uint16_t)hk;")]
PATCHES["l1noatom"] = [("hm_kernels.hip", "        if (cnt[q]) gpos[q] = atomicAdd(&a.fill[hm_l1i(d, sh)], cnt[q]);",
                        "        if (cnt[q]) gpos[q] = 0;")]
# k_small_pairs timing builds: no cursor atomic (a made-up base), no cell
# stores, no emit pass at all (profiles/r6/small_pairs_atomics_ab.jsonl has
# the round-6 per-wave-reservation results, incl. sharded and non-returning
# cursor atomics)
PATCHES["spnoatom"] = [("hm_kernels.hip", "s_base = btotal ? atomicAdd(a.out.cursor, (unsigned long long)btotal) : 0ull;",
                        "s_base = (unsigned long long)(kb & 0xFFFFFu) * 96u * HM_SPP_WAVES * 64u;")]
PATCHES["stamps7noatom"] = PATCHES["spnoatom"]
PATCH_DEFINES["stamps7noatom"] = ["HM_STAMPS=7"]
# k_small_pairs held to 8 waves per SIMD (<= 96 SGPRs), with 16 rows a round (LDS for 8 blocks)
PATCHES["sp8w16"] = [("hm_kernels.hip", "__global__ __launch_bounds__(64 * NWB) void k_small_pairs(HmAggArgs a)",
                      "__global__ __launch_bounds__(64 * NWB) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_small_pairs(HmAggArgs a)")]
PATCH_DEFINES["sp8w16"] = ["HM_SPP_ROWS=16"]
PATCHES["spnostore"] = [("hm_kernels.hip", """            const uint64_t pos = q + hm_mbcnt(bal);
            if (pos < a.out.capacity) {""", """            const uint64_t pos = q + hm_mbcnt(bal);
            if (pos == 0x123456789ull) {""")]
# levels 2.. always on the spread plan (3 zooms per level) when no tile is hot
PATCHES["spreadall"] = [("hm_api.cpp", "spread_replan(ctx->host_aux, F, (double)n, zb, zs, &L, ctx->spread_min_keys, true);",
                         "spread_replan(ctx->host_aux, F, (double)n, zb, zs, &L, ctx->spread_min_keys, false);")]
# k_l1_fast at one block per CU (an 80 KB LDS pad): K1's sensitivity to occupancy
PATCHES["l1occ1"] = [("hm_kernels.hip", """    __shared__ uint32_t s_over;
    /* the polynomial table plus one poison row""", """    __shared__ uint32_t s_over;
    __shared__ uint32_t occpad[20480];
    if (a.n == -12345) occpad[threadIdx.x] = 1;
    /* the polynomial table plus one poison row""")]
# the exchange's bucket merge (k_mb_merge2): no LDS insertion atomics (each
# key stored at its home slot), or no output stores
PATCHES["mb2noins"] = [("hm_merge.hip", """                        const unsigned long long o =
                            atomicCAS(&tk[sl], (unsigned long long)HMS_EMPTY, (unsigned long long)k[j]);""",
                        """                        tk[sl] = k[j];
                        const unsigned long long o = k[j];""")]
PATCHES["mb2nowrite"] = [("hm_merge.hip", """                    if (q < a.cap) {
                        a.keys_out[q] = tk[sl];
                        a.counts_out[q] = tc[sl];
                    }""", """                    if (q == 0x123456789ull) {
                        a.keys_out[q] = tk[sl];
                        a.counts_out[q] = tc[sl];
                    }""")]
PATCHES["mb2nocur"] = [("hm_merge.hip", "if (lane == 63) sbase = inc ? atomicAdd(a.cursor, (unsigned long long)inc) : 0ull;",
                        "if (lane == 63) sbase = (uint64_t)b * 1024u;")]
PATCHES["mb2loadonly"] = [("hm_merge.hip", """                for (int j = 0; j < 4; j++) {
                    if (k[j] == HMS_EMPTY) continue;
                    const uint64_t h = hms_hash(k[j]);""", """                for (int j = 0; j < 4; j++) {
                    if (k[j] != 0x1234567ull) continue;
                    const uint64_t h = hms_hash(k[j]);""")]
# one-sweep radix passes without the decoupled look-back (timing only: wrong offsets)
PATCHES["rxnolb"] = [("hm_general.hip", """        for (int64_t p = (int64_t)tile - 1; p >= 0;) {
            const uint64_t wv = __hip_atomic_load(a.tstat + (uint64_t)p * 256 + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""",
                      """        for (int64_t p = (int64_t)tile - 1; p >= 0 && p == 0x7FFFFFFFFFFF;) {
            const uint64_t wv = __hip_atomic_load(a.tstat + (uint64_t)p * 256 + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""")]
# k_aggregate: multi-item buckets without their global histogram adds (timing only)
PATCHES["agnoslot"] = [("hm_kernels.hip", "            if (i < ncell && x[k]) atomicAdd(&g[i], x[k]);",
                        "            if (i < ncell && x[k] == 0xFFFFFFFFu) atomicAdd(&g[i], x[k]);")]
# hm_count's emit reservations without the cursor atomic (timing only)
PATCHES["emitnocur"] = [("hm_kernels.hip", "if (lane == NW - 1) *sbase = incl ? atomicAdd(o.cursor, (unsigned long long)incl) : 0ull;",
                         "if (lane == NW - 1) *sbase = (uint64_t)(hm_block_id() & 4095u) * 16384u;"),
                        ("hm_kernels.hip", "if (threadIdx.x == 0) *sbase = atomicAdd(o.cursor, (unsigned long long)tot);",
                         "if (threadIdx.x == 0) *sbase = (uint64_t)(hm_block_id() & 4095u) * 16384u;")]
# the route's scatter without its record stores
PATCHES["xrnostore"] = [("hm_merge.hip", """            if (OUT == 0) {
                hm_rec_put(a.rec_out + 5 * q, sk[i], (uint32_t)sc[i]);""", """            if (OUT == 0) {
                if (q == 0x123456789ull) hm_rec_put(a.rec_out + 5 * q, sk[i], (uint32_t)sc[i]);""")]
# hm_emit_cells (k_aggregate's pyramid emission) without its cell stores (timing only)
PATCHES["agnoemit"] = [("hm_kernels.hip", """        if (nz && pos < o.capacity) {
            o.keys[pos] = k;""", """        if (nz && pos == 0x123456789ull) {
            o.keys[pos] = k;""")]
# K1 phase-lockstep probe: the first round's second block of a CU starts ~16 us
# late, so the two resident blocks alternate load and compute phases from then on
PATCHES["l1stag256"] = [("hm_kernels.hip", """    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);""", """    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);
    if (blockIdx.x >= 256 && blockIdx.x < 512)
        for (int z = 0; z < 5; z++) __builtin_amdgcn_s_sleep(127);""")]
PATCHES["l1stagodd"] = [("hm_kernels.hip", """    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);""", """    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);
    if (blockIdx.x < 512 && (blockIdx.x & 1))
        for (int z = 0; z < 5; z++) __builtin_amdgcn_s_sleep(127);""")]
PATCHES["l1stagall"] = [("hm_kernels.hip", """    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);""", """    const int64_t base = (a.tile0 + (int64_t)blockIdx.x) * HM_T1;
    HM_STAMP_M(4, 0);
    if (blockIdx.x < 512)
        for (int z = 0; z < (int)(blockIdx.x & 7); z++) __builtin_amdgcn_s_sleep(127);""")]
# k_aggregate's count without any wave merging: one plain LDS atomic per key
PATCHES["agplain"] = [("hm_kernels.hip", """            if (HM_AG_FAST)
                hm_lds_count_fast(grid, dummy + (uint32_t)hm_lane(), sl(k), v);
            else
                hm_lds_count(grid, dummy, sl(k), v);""", """            atomicAdd(&grid[v ? sl(k) : dummy + (uint32_t)hm_lane()], 1u);""")]
# k_small_emit's pair path (<= 32-key buckets, the skew cloud's background) without its cell stores (timing only)
PATCHES["emnostore"] = [("hm_kernels.hip", """                        if (p < a.out.capacity) {
                            a.out.keys[p] = hm_cell_key(a.Z - l, coord, s, idx);""", """                        if (p == 0x123456789ull) {
                            a.out.keys[p] = hm_cell_key(a.Z - l, coord, s, idx);""")]
# compile-time macros added to a patched build


def build(names):
    import shutil
    import tempfile

    from heatmap_amd import build as b

    for n in names:
        out = os.path.join(VDIR, "lib_%s.so" % n)
        if n.startswith("git-"):
            # the sources of a commit ("git-<rev>"): an A/B against a committed state
            tmp = tempfile.mkdtemp()
            subprocess.run("git -C %s archive %s heatmap_amd/csrc include | tar -x -C %s" % (REPO, n[4:], tmp),
                           shell=True, check=True)
            b.build(force=True, verbose=False, out=out, csrc=os.path.join(tmp, "heatmap_amd", "csrc"))
            shutil.rmtree(tmp)
        elif n in PATCHES:
            tmp = tempfile.mkdtemp()
            src = os.path.join(tmp, "pkg", "csrc")       # keeps "../../include/" valid
            shutil.copytree(b.CSRC, src)
            shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
            for f, old, new in PATCHES[n]:
                p = os.path.join(src, f)
                t = open(p).read()
                assert old in t, (n, f, old)
                open(p, "w").write(t.replace(old, new))
            b.build(force=True, verbose=False, out=out, csrc=src, defines=PATCH_DEFINES.get(n, []))
            shutil.rmtree(tmp)
        else:
            b.build(force=True, verbose=False, out=out, defines=VARIANTS[n])
        print("built", out, flush=True)


def one(name, points, steps, zmax, zmin=0):
    if name != "main":     # "main": the in-tree library heatmap_amd/_lib/libheatmap_amd.so
        os.environ["HM_LIB_PATH"] = os.path.join(VDIR, "lib_%s.so" % name)
    import numpy as np
    import torch

    from heatmap_amd import device

    lat = torch.empty(points, dtype=torch.float64, device="cuda")
    lon = torch.empty(points, dtype=torch.float64, device="cuda")
    device.synth(os.environ.get("HM_KIND", "hotspots"), lat, lon)
    bufs = device.CountBuffers(64 << 20)
    ctx = device.context(0)
    m, bufs = device.count_device(lat, lon, None, zmin, zmax, 0, buffers=bufs)
    torch.cuda.synchronize()
    st = []
    t0 = time.perf_counter()
    for _ in range(steps):
        m, bufs = device.count_device(lat, lon, None, zmin, zmax, 0, buffers=bufs)
        ls = ctx.last_stats()[1]
        st.append(list(ls[:4]) + [ls[6], ls[5]])   # stage times, hot tiles, level-1 re-runs
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    tot = int(bufs.counts[:m].sum().item())
    # cell-for-cell parity when the golden digest of this cloud exists
    kind = os.environ.get("HM_KIND", "hotspots")
    gname = "%s_%de%d_z%d-%d" % (kind, int(str("%e" % points)[0]), len(str(points)) - 1, zmin, zmax)
    gd = json.load(open(os.path.join(REPO, "tests", "golden", "big_digests.json"))).get(gname)
    digest = None
    if gd is not None and gd["n"] == points and gd["zmin"] == zmin:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from digest import device_digest

        digest = device_digest(torch, bufs.keys[:m], bufs.counts[:m]) == gd["digest"]
    print(json.dumps({"variant": name, "ms": dt * 1e3, "gpts": points / dt / 1e9, "cells": m,
                      "check": tot == points * (zmax - zmin + 1), "digest_ok": digest, "kind": kind,
                      "stage_us": [round(x, 1) for x in np.mean(np.array(st), axis=0)]}), flush=True)


def merge_one(name, points, steps):
    """The exchange at world size 1 (the rehearsal's route + merge, no RCCL):
    per-call times of hm_cells_route_pieces and hm_cells_merge_pieces over the
    cells of one count; the owned cells must be the counted ones."""
    if name != "main":
        os.environ["HM_LIB_PATH"] = os.path.join(VDIR, "lib_%s.so" % name)
    import torch

    from heatmap_amd import _lib, device, multigpu

    lat = torch.empty(points, dtype=torch.float64, device="cuda")
    lon = torch.empty(points, dtype=torch.float64, device="cuda")
    device.synth("hotspots", lat, lon)
    m, bufs = device.count_device(lat, lon, None, 0, 18)
    del lat, lon
    keys, counts = bufs.keys[:m].clone(), bufs.counts[:m].clone()
    ops = multigpu.DeviceOps(0)
    bits = multigpu.route_bits(1)
    ok, tr, tm = True, [], []
    for it in range(steps + 1):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        _, parts, sizes = ops.route_pieces(keys, counts, 1, 10, bits, _lib.HM_CELLS_REC10)
        e[1].record()
        pieces = sizes.cpu()[:, 2:2 + (1 << bits)].tolist()
        uk, uc = ops.merge_pieces([(parts[0][0], None, 0)], pieces, bits, _lib.HM_CELLS_REC10)
        e[2].record()
        torch.cuda.synchronize()
        if it:
            tr.append(e[0].elapsed_time(e[1]))
            tm.append(e[1].elapsed_time(e[2]))
        sp = (keys >> 58) > 10
        ok = ok and uk.numel() == int(sp.sum()) and int(uc.sum()) == int(counts[sp].sum())
    tr.sort()
    tm.sort()
    print(json.dumps({"variant": name, "route_ms": tr[len(tr) // 2], "merge_ms": tm[len(tm) // 2], "cells": m,
                      "lb": os.environ.get("HM_MERGE_LB", "1"), "ok": ok}), flush=True)


def main():
    cmd = sys.argv[1]
    names = sys.argv[2:] or ["base"]
    if cmd == "build":
        build(names)
    elif cmd == "run":
        for n in names:
            r = subprocess.run([sys.executable, __file__, "one", n], timeout=300)
            if r.returncode != 0:
                print(json.dumps({"variant": n, "error": r.returncode}), flush=True)
                break
    elif cmd == "mrun":
        for n in names:
            r = subprocess.run([sys.executable, __file__, "mone", n], timeout=300)
            if r.returncode != 0:
                print(json.dumps({"variant": n, "error": r.returncode}), flush=True)
                break
    elif cmd == "mone":
        merge_one(names[0], int(float(os.environ.get("HM_POINTS", "1.25e9"))), int(os.environ.get("HM_STEPS", "5")))
    elif cmd == "one":
        one(names[0], int(float(os.environ.get("HM_POINTS", "1e9"))), int(os.environ.get("HM_STEPS", "3")),
            int(os.environ.get("HM_ZMAX", "18")), int(os.environ.get("HM_ZMIN", "0")))


if __name__ == "__main__":
    main()
