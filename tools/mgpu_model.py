"""Multi-GPU round-time model from one GPU (experiment tool).

    python tools/mgpu_model.py run   <n> <topology> <algorithm> <W> <rounds>
    python tools/mgpu_model.py model <trace dir> <n> <topology> <algorithm> <W> <rounds> [out.json]

`run` is the workload: W in-process virtual ranks on one device
(GP_FLAG_VIRTUAL_RANKS -- the same slab plan, kernels and exchange order as W
processes over RCCL, with device copies as the transport), advanced to steady
state (push-sum: every node active), then `rounds` timed rounds.  Run it under
`rocprofv3 --kernel-trace`.

`model` reads that trace.  Rounds are cut after every group of W
`k_finalize_post` dispatches (the last kernels of a multi-rank round); inside a
round the k-th dispatch of a kernel launched once per slab belongs to slab k.
Per rank: the sum of its kernels (round kernel, pack / unpack or the full
topology's binning passes, finalize) = what that rank's GPU computes per round
at world W (each slab ran alone on the whole device, as it would on its own
GPU).  Device-copy kernels are the virtual transport and are dropped; in their
place the exchange is modelled from the bytes RCCL moves per round -- the
fixed-capacity buffers of setup_exchange (restated in tests/test_multigpu_plan.py)
and the halo planes -- over point-to-point xGMI links (one link per rank pair
on an 8-GPU node) at the assumed per-direction link rates, plus an assumed
latency per RCCL group and for the 4 x u64 bookkeeping all-reduce.  Nothing here
is a measured multi-GPU number.
"""
import csv
import glob
import json
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINK_GBPS = (64.0, 128.0)   # assumed achieved RCCL send/recv rate per xGMI link and direction
GROUP_LAT_MS = 0.020        # assumed latency of one grouped send/recv
ALLREDUCE_LAT_MS = 0.015    # assumed latency of the 4 x u64 all-reduce


def run(n, topo, alg, W, rounds):
    import time

    from gossipprotocol_amd import Simulation
    # the experiments build (GP_* overrides) when asked for, as tools/perf_round.py
    exp = bool(os.environ.get("GOSSIP_HIP_LIB_EXPERIMENT") or os.environ.get("GP_EXP"))
    s = Simulation(n, topo, alg, virtual_ranks=W, experimental=exp)
    P = s.population
    pre = 0
    t = time.perf_counter()
    if alg == "push-sum":
        while s.info().active < P and pre < 3000:
            pre += len(s.step(8))
    else:
        pre += len(s.step(40))
    s.sync()
    tp = time.perf_counter() - t
    t = time.perf_counter()
    got = s.step(rounds)
    s.sync()
    wall = time.perf_counter() - t
    print(json.dumps({"n": n, "topology": topo, "algorithm": alg, "W": W, "P": P, "preroll_rounds": pre,
                      "preroll_s": tp, "rounds": len(got), "wall_ms_per_round_virtual": wall * 1e3 / max(1, len(got))}),
          flush=True)
    s.close()


def per_slab_names(groups, short):
    return {short(name) for grp in groups for name, _ in grp}


def pair_bytes(n, topo, alg, W, halves=1, lists=True, halo_compact=False):
    """Bytes rank a sends rank b per round (fixed-capacity buffers incl. their 16-B count
    headers; full push-sum: `halves` regions, one per half of a's senders) and the halo
    bytes per neighbouring pair and direction (push-sum since round 5: the plane's direction
    bytes + HALO_CAP = 256 (s, w) slots per 1024-node chunk, gp_xchg.hpp)."""
    from tests.multirank_emu import full_bin_multi_cap, full_bin_multi_s1, full_region, resolve, slab_bounds
    from tests.test_multigpu_plan import cap_of, imp3d_pair_stats
    P, _, g = resolve(n, topo)
    push = alg == "push-sum"

    def xbuf(cap):
        return 0 if cap <= 0 else 16 + ((cap * 4 + 15) & ~15) + (16 * cap if push else 0)

    B = [[0] * W for _ in range(W)]
    halo = 0
    if topo == "full":
        # push-sum since round 6: per region, the destination's coarse bins (FbBins: counts,
        # sender ids, payloads at a fixed capacity per bin, gp_fullbin.hip)
        from tests.test_multigpu_plan import fb_bins_bytes
        bounds, _ = slab_bounds(P, g, topo, W)
        s1 = full_bin_multi_s1(bounds)
        nb = [-(-(bounds[b + 1] - bounds[b]) // (1 << s1)) for b in range(W)]
        for a in range(W):
            na = bounds[a + 1] - bounds[a]
            for b in range(W):
                if b != a:
                    for h in range(halves):
                        r0, r1 = full_region(na, halves, h)
                        B[a][b] += fb_bins_bytes(nb[b], full_bin_multi_cap(r1 - r0, s1, P))
    else:
        bounds, H = slab_bounds(P, g, topo, W)
        halo = H * (1 + (16 if push else 0))
        if push and halo_compact:
            halo = H + (H + 1023) // 1024 * 256 * 16
        if topo == "Imp3D":
            _, mu, _ = imp3d_pair_stats(P, g, W)
            for a in range(W):
                na = bounds[a + 1] - bounds[a]
                nt = na // 1024 + 1
                for b in range(W):
                    if b == a:
                        continue
                    if push and lists:
                        # sender-ordered lists (round 5): per region the header words (16 B per 64
                        # list entries, a tile's segment padded to 64: ~half a word per tile) and the
                        # message slots (16 B each, capacity per region)
                        edges = na * (bounds[b + 1] - bounds[b]) / (P - 1)
                        B[a][b] = int(16 * (edges / 64 + nt / 2)) + sum(16 * cap_of(mu[a, b] / halves)
                                                                        for _ in range(halves))
                    elif not push and lists:
                        # gossip (column kernel) since round 5: one bit per edge a -> b, chunks
                        # padded to 1024 bits
                        edges = na * (bounds[b + 1] - bounds[b]) / (P - 1)
                        B[a][b] = int(math.ceil(edges / 1024) * 128)
                    else:  # {slot, (s, w)} buffers (round 4) / gossip counts
                        B[a][b] = sum(xbuf(cap_of(mu[a, b] / halves)) for _ in range(halves))
    return P, bounds, B, halo


def model(tdir, n, topo, alg, W, rounds, out=None):
    rows = []
    for f in glob.glob(tdir + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    groups, cur, nfin = [], [], 0
    for r in rows:
        name = r["Kernel_Name"]
        cur.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
        if "k_finalize_post" in name:
            nfin += 1
            if nfin == W:
                groups.append(cur)
                cur, nfin = [], 0
    groups = groups[-rounds:]
    if not groups:
        raise SystemExit("no multi-rank rounds in the trace")
    short = lambda k: k.split("(")[0].replace("void ", "").replace("gp::", "")  # noqa: E731
    per_slab, glob_k, copy_ms = {}, {}, []
    rank_ms = [[] for _ in range(W)]
    for grp in groups:
        by = {}
        for name, ms in grp:
            by.setdefault(name, []).append(ms)
        tr = [0.0] * W
        cp = 0.0
        for name, v in by.items():
            if "rocclr_copy" in name:
                cp += sum(v)
            elif len(v) == W or (len(v) % W == 0 and ("k_ps_tile" in name or "k_fb_" in name)):
                # (region-by-region rounds: the round kernel once per region and slab, slab k's
                # launches at k, W + k, ...)
                vs = [sum(v[h * W + k] for h in range(len(v) // W)) for k in range(W)]
                per_slab.setdefault(short(name), []).append(vs)
                for k in range(W):
                    tr[k] += vs[k]
            elif "fill" not in name:  # (memsets: counters, on every rank)
                glob_k.setdefault(short(name), []).append(sum(v))
                for k in range(W):
                    tr[k] += sum(v) / max(1, len(v)) * (len(v) / W)
            else:
                for k in range(W):
                    tr[k] += sum(v) / W
        copy_ms.append(cp)
        for k in range(W):
            rank_ms[k].append(tr[k])
    # push-sum runs its exchange in two halves overlapped with the send / coarse passes
    # (full, gp_api.hip launch_round_full_multi) or the pack / unpack (Imp3D, exchange):
    # those kernels appear twice per slab
    halves = 2 if alg == "push-sum" and topo in ("full", "Imp3D") else 1
    if alg == "push-sum" and topo == "Imp3D":  # round 5: XREGIONS list regions (k_list_pack per region and slab)
        npk = [sum(1 for name, _ in grp if short(name) == "k_list_pack") for grp in groups]
        if npk and npk[-1] and npk[-1] % W == 0:
            halves = npk[-1] // W
    # (Imp3D push-sum since round 5: k_list_pack per region, no unpack -- the round kernel reads the
    # received lists in place; full push-sum since round 6: no send / coarse pass, see below)
    first_k, second_k = ("k_fbm_send", "k_fbm_coarse") if topo == "full" else ("k_list_pack", None)
    # a round-4 build (A/B runs): {slot} / {count} buffers with an unpack pass
    legacy = topo != "full" and any("k_unpack" in k for k in per_slab_names(groups, short))
    if legacy:
        first_k, second_k = "k_pack", "k_unpack"
    # compacted halo planes (round 5): k_halo_pack in the trace
    hc = any("k_halo" in k for k in per_slab_names(groups, short))
    P, bounds, B, halo = pair_bytes(n, topo, alg, W, halves, lists=not legacy, halo_compact=hc)
    kern = {k: [statistics.mean(x[s] for x in v) for s in range(W)] for k, v in per_slab.items()}
    comp = [statistics.mean(v) for v in rank_ms]
    t_comp = max(comp)
    piped = None
    # region-by-region rounds (gp_api.hip launch_round_regions): per rank the round kernel of
    # region h, then region h's pack; region h's transfer after both, overlapping region h + 1
    rk_name = next((nm for nm in per_slab_names(groups, short) if nm.startswith("k_ps_tile")), None)
    nreg = 0
    if rk_name and alg == "push-sum" and topo == "Imp3D":
        nk = sum(1 for name, _ in groups[-1] if short(name) == rk_name)
        nreg = nk // W if nk % W == 0 and nk > W else 0
    regions = None
    if nreg:
        kr, pr = [], []
        for grp in groups:
            kv = [ms for name, ms in grp if short(name) == rk_name]
            pv = [ms for name, ms in grp if short(name) == "k_list_pack"]
            if len(kv) == nreg * W and len(pv) == nreg * W:
                kr.append(kv)
                pr.append(pv)
        if kr:
            K = [[statistics.mean(x[h * W + k] for x in kr) for h in range(nreg)] for k in range(W)]
            Pk = [[statistics.mean(x[h * W + k] for x in pr) for h in range(nreg)] for k in range(W)]
            regions = {"kernel_region_ms": [round(max(K[k][h] for k in range(W)), 4) for h in range(nreg)],
                       "pack_region_ms": [round(max(Pk[k][h] for k in range(W)), 4) for h in range(nreg)],
                       "K": K, "P": Pk}
    # full push-sum (round 6, gp_api.hip launch_round_full_multi): per rank the splits of every
    # region, then region by region the fold, whose messages travel (region h's transfer after
    # its fold, in order on the link) while the next region folds
    fused = None
    if topo == "full" and alg == "push-sum":
        sv, fv = [], []
        for grp in groups:
            a_ = [ms for name, ms in grp if short(name).startswith("k_fb_split")]
            b_ = [ms for name, ms in grp if short(name).startswith("k_fb_fold")]
            if len(a_) == halves * W and len(b_) == halves * W:
                sv.append(a_)
                fv.append(b_)
        if fv:
            Sp = [[statistics.mean(x[h * W + k] for x in sv) for h in range(halves)] for k in range(W)]
            Fo = [[statistics.mean(x[h * W + k] for x in fv) for h in range(halves)] for k in range(W)]
            fused = {"split_region_ms": [round(max(Sp[k][h] for k in range(W)), 4) for h in range(halves)],
                     "fold_region_ms": [round(max(Fo[k][h] for k in range(W)), 4) for h in range(halves)],
                     "S": Sp, "F": Fo}
    if halves >= 2 and not regions and not fused:
        # per rank: send half 0, half 1; coarse half 0, half 1 (dispatch order), the rest
        hk = {}
        for grp in groups:
            by = {}
            for name, ms in grp:
                by.setdefault(short(name), []).append(ms)
            for nm in (first_k, second_k):
                v = by.get(nm, [])
                if nm and len(v) == halves * W:
                    hk.setdefault(nm, []).append(v)
        if len(hk.get(first_k, [])) and (second_k is None or len(hk.get(second_k, []))):
            s_h = [[statistics.mean(x[h * W + k] for x in hk[first_k]) for k in range(W)] for h in range(halves)]
            c_h = ([[statistics.mean(x[h * W + k] for x in hk[second_k]) for k in range(W)] for h in range(halves)]
                   if second_k else [[0.0] * W for _ in range(halves)])
            piped = {"send_half_ms": [max(v) for v in s_h], "coarse_half_ms": [max(v) for v in c_h],
                     "rest_ms": max(comp[k] - sum(s_h[h][k] + c_h[h][k] for h in range(halves)) for k in range(W))}
    res = {"workload": f"{alg} {topo} n={n} P={P}", "W": W, "rounds_measured": len(groups),
           "per_slab_kernel_ms": {k: [round(x, 4) for x in v] for k, v in kern.items()},
           "global_kernel_ms": {k: round(statistics.mean(v), 4) for k, v in glob_k.items()},
           "virtual_copy_ms": round(statistics.mean(copy_ms), 4),
           "rank_compute_ms": [round(x, 4) for x in comp],
           "pair_bytes_max": max(max(r) for r in B), "bytes_out_per_rank_max": max(sum(r) for r in B),
           "halo_bytes_per_direction": halo, "assumptions": {
               "link_gbps_per_direction": LINK_GBPS, "group_latency_ms": GROUP_LAT_MS,
               "allreduce_latency_ms": ALLREDUCE_LAT_MS, "topology": "one xGMI link per rank pair (8-GPU node)"},
           "model": [], "pipelined_halves": piped,
           "round_regions": ({k: v for k, v in regions.items() if k in ("kernel_region_ms", "pack_region_ms")}
                             if regions else None),
           "full_fused_regions": ({k: v for k, v in fused.items() if k in ("split_region_ms", "fold_region_ms")}
                                  if fused else None)}
    for bw in LINK_GBPS:
        # the busiest link: a pair's buffer plus, between slab neighbours, the halo plane
        link = 0.0
        for a in range(W):
            for b in range(W):
                if a != b:
                    link = max(link, B[a][b] + (halo if abs(a - b) == 1 else 0))
        t_x = link / (bw * 1e9) * 1e3 + (GROUP_LAT_MS if link else 0.0) * halves
        serial = t_comp + t_x + ALLREDUCE_LAT_MS
        overlap = max(t_comp, t_x) + ALLREDUCE_LAT_MS
        if fused:  # as scheduled, per rank: S_0 S_1 F_0 F_1; x_h after F_h, in order on the link
            Sp, Fo = fused["S"], fused["F"]
            xh = t_x / halves
            worst = 0.0
            for k in range(W):
                t = sum(Sp[k])
                x_end = 0.0
                for h in range(halves):
                    t += Fo[k][h]
                    x_end = max(x_end, t) + xh
                worst = max(worst, max(t, x_end) + comp[k] - sum(Sp[k]) - sum(Fo[k]))
            overlap = worst + ALLREDUCE_LAT_MS
        elif regions:  # as scheduled, per rank: K_0 P_0 K_1 P_1 ...; x_h after P_h, in order on the link
            K, Pk = regions["K"], regions["P"]
            xh = t_x / nreg
            worst = 0.0
            for k in range(W):
                t = x_end = 0.0
                for h in range(nreg):
                    t += K[k][h] + Pk[k][h]
                    x_end = max(x_end, t) + xh
                worst = max(worst, max(t, x_end) + comp[k] - sum(K[k]) - sum(Pk[k]))
            overlap = worst + ALLREDUCE_LAT_MS
        elif piped:  # as scheduled: x_h after send_h / pack_h, coarse_h / unpack_h after x_h (one exchange stream)
            sh, ch = piped["send_half_ms"], piped["coarse_half_ms"]
            nh = len(sh)
            xh = t_x / nh
            t_send = x_end = 0.0
            for h in range(nh):  # packs back to back on the compute stream, transfers in order on the exchange stream
                t_send += sh[h]
                x_end = max(x_end, t_send) + xh
            if nh == 2:  # full topology: the coarse pass of half 0 overlaps half 1's transfer
                x0_end = sh[0] + xh
                c_end = max(max(sh[0] + sh[1], x0_end) + ch[0], x_end) + ch[1]
            else:
                c_end = x_end + sum(ch)
            overlap = c_end + piped["rest_ms"] + ALLREDUCE_LAT_MS
        res["model"].append({"link_gbps": bw, "exchange_ms": round(t_x, 4), "round_ms_serial": round(serial, 4),
                             "round_ms_as_scheduled": round(overlap, 4) if piped or regions or fused else round(serial, 4),
                             "exchange_share_serial": round(t_x / serial, 3), "round_ms_overlapped": round(overlap, 4),
                             "node_updates_per_s_serial": P / (serial * 1e-3),
                             "node_updates_per_s_overlapped": P / (overlap * 1e-3)})
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


def main():
    if sys.argv[1] == "run":
        run(int(sys.argv[2]), sys.argv[3], sys.argv[4], int(sys.argv[5]), int(sys.argv[6]))
    else:
        model(sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5], int(sys.argv[6]), int(sys.argv[7]),
              sys.argv[8] if len(sys.argv) > 8 else None)


if __name__ == "__main__":
    main()
