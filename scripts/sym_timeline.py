"""Timeline of one faml_sym_repulse launch at C4 (diagnostics, GE_SYM_STAMPS).

Builds the C4 level-0 plan as bench.py does, runs ITERS iterations with the
stamping kernel variant, and summarises the last launch's per-unit stamps
(ge_sym.hpp: take / first hand-over / end / spin ticks of s_memrealtime, 100 MHz):
launch span, wave occupancy over time, parked share, the tail after the queue
drained, and the critical aggregates' chains.  With STAMPS_ONLY=path it only
analyses an existing dump.
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    raw = open(path, "rb").read()
    nunits, words, blocks, threads = np.frombuffer(raw[:16], dtype=np.int32)
    units = np.frombuffer(raw[16:16 + 16 * nunits], dtype=np.int32).reshape(nunits, 4)
    st = np.frombuffer(raw[16 + 16 * nunits:], dtype=np.int64).reshape(nunits, words)
    return units, st, int(blocks) * int(threads) // 64


def analyse(path):
    units, st, waves = load(path)
    t0 = st[:, 0].min()
    take, first, end, spin = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, (st[:, 2] - t0) / 100.0, st[:, 3] / 100.0
    span = end.max()  # microseconds
    dur = end - take
    busy = dur - spin
    out = {"units": int(len(units)), "waves": waves, "span_ms": span / 1e3,
           "wave_time_share_spinning": float(spin.sum() / (waves * span)),
           "wave_time_share_busy": float(busy.sum() / (waves * span)),
           "wave_time_share_idle_no_unit": float(1.0 - dur.sum() / (waves * span)),
           "queue_drained_ms": float(take.max() / 1e3),
           "tail_after_drain_ms": float((span - take.max()) / 1e3),
           "park_before_first_tile_share": float((first - take).sum() / (waves * span))}
    # waves holding a unit / computing (not spinning: approximated by [first, end]) per time bin
    bins = np.linspace(0, span, 41)
    hold = np.zeros(40)
    comp = np.zeros(40)
    for a, b, f in zip(take, end, first):
        for arr, lo in ((hold, a), (comp, f)):
            i0 = np.searchsorted(bins, lo, "right") - 1
            i1 = np.searchsorted(bins, b, "right") - 1
            for i in range(max(i0, 0), min(i1, 39) + 1):
                ov = min(b, bins[i + 1]) - max(lo, bins[i])
                if ov > 0:
                    arr[i] += ov / (bins[i + 1] - bins[i])
    out["holding_waves_by_2.5pct"] = [round(x) for x in hold]
    out["computing_waves_by_2.5pct"] = [round(x) for x in comp]
    # per aggregate: chain length = its last end - its first take
    aggs = {}
    for q in range(len(units)):
        a = int(units[q, 0])
        e = aggs.setdefault(a, [1e18, 0.0, 0, 0.0, int(units[q, 3])])
        e[0] = min(e[0], take[q])
        e[1] = max(e[1], end[q])
        e[2] += 1
        e[3] += spin[q]
    crit = sorted(aggs.items(), key=lambda kv: -kv[1][1])[:8]
    out["latest_aggregates"] = [{"agg": a, "tiles": v[2], "kind": v[4], "first_take_ms": v[0] / 1e3,
                                 "last_end_ms": v[1] / 1e3, "spin_ms_sum": v[3] / 1e3} for a, v in crit]
    # per-tile time of the sweeps: duration / tiles processed
    kind = units[:, 3] & 15  # ge_sym.hpp unit_word: kind | band first tile << 4 | band end << 18
    sw = kind == 0
    out["sweep_unit_us_median"] = float(np.median(dur[sw])) if sw.any() else None
    for name, k in (("sweep", 0), ("rows", 1), ("pre", 3)):
        sel = kind == k
        if sel.any():
            out[f"{name}_units"] = {"count": int(sel.sum()), "dur_us_median": float(np.median(dur[sel])),
                                    "dur_ms_sum": float(dur[sel].sum() / 1e3),
                                    "spin_ms_sum": float(spin[sel].sum() / 1e3),
                                    "last_end_ms": float(end[sel].max() / 1e3),
                                    "first_take_ms": float(take[sel].min() / 1e3)}
    # per SIMD (HW_ID bits: wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13; XCC_ID low bits)
    hw = st[:, 4]
    simd = (st[:, 5] & 0xF) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15) * 16 + ((hw >> 4) & 3)
    per = {}
    for k, b in zip(simd, busy):
        per[int(k)] = per.get(int(k), 0.0) + b
    v = np.array(list(per.values())) / span
    out["simds_seen"] = int(len(per))
    out["busy_waves_per_simd"] = {"min": float(v.min()), "median": float(np.median(v)), "max": float(v.max())}
    return out


def main():
    if os.environ.get("STAMPS_ONLY"):
        print(json.dumps(analyse(os.environ["STAMPS_ONLY"])))
        return
    import torch
    sys.path.insert(0, os.path.join(REPO, "graph-embed_amd", "py"))
    import ge_amd as ge
    path = os.environ.setdefault("GE_SYM_STAMPS", os.path.join(REPO, "gpurun_out", "sym_stamps.bin"))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    n, draws, dim, iters = 10_000_000, 80_000_000, 3, int(os.environ.get("ITERS", "2"))
    ctx = ge.Context(0)
    L = ctx.rmat_csr(n, draws, seed=12345, lcc=True)
    PT = ctx.partition(L, 0.125)[0]
    m = PT[2]
    n0 = len(L[0]) - 1
    vA = ge.vertex_of(PT)
    dev = torch.device("cuda:0")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = dict(ip=T(L[0]), ix=T(L[1]), dx=T(L[2]), pip=T(PT[0]), pix=T(PT[1]), vA=T(vA),
             cA=T(ge.uniform_stream(7, m * dim)), rA=T(0.01 + 0.19 * (ge.uniform_stream(8, m) + 1) / 2),
             init=T(ge.uniform_stream(5, n0 * dim)))
    X = torch.zeros((n0, dim), dtype=torch.float64, device=dev)
    # SHARES=N: also every rank's share of an N-GPU deal (scale_sim.py), one dump each
    runs = [(1, 0)] + [(int(N), r) for N in os.environ.get("SHARES", "").split(",") if N
                       for r in range(int(N))]
    for N, r in runs:
        aggs = None
        if N > 1:
            aggs = np.flatnonzero(ge.assign_aggregates(PT, L[0], N) == r).astype(np.int32)
        dump = path if N == 1 else f"{path}.N{N}r{r}"
        os.environ["GE_SYM_STAMPS"] = dump
        if os.path.exists(dump):
            os.remove(dump)
        p = ge.FamlPlan(ctx, n0, d["ip"].data_ptr(), d["ix"].data_ptr(), d["dx"].data_ptr(),
                        PT[0], d["pip"].data_ptr(), d["pix"].data_ptr(), d["vA"].data_ptr(), dim,
                        iterations=iters, aggs=aggs)
        p.set_profiling(True)
        p.run(d["cA"].data_ptr(), d["rA"].data_ptr(), d["init"].data_ptr(), X.data_ptr())
        ctx.sync()
        rep_ms, _, _ = p.repulse_ms()
        p.close()
        res = analyse(dump) if os.path.exists(dump) else {"units": 0}
        res.update({"N": N, "rank": r, "repulse_ms_events": rep_ms})
        print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
