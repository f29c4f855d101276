#!/usr/bin/env python3
"""Turn a tools/collect_profiles.sh run (gpurun_out/profiles) into the committed profiles/:
kernel-stat tables (markdown), PMC-derived metrics, and the raw rocprofv3 stats CSVs."""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys

SRC = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "pmc-ab" else "gpurun_out/profiles"
DST = sys.argv[2] if len(sys.argv) > 2 else "profiles"


def stats_table(name: str, limit: int = 12) -> str:
    path = os.path.join(SRC, name, "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(path)))
    out = [f"| kernel | calls | avg µs | total ms | % |", "|---|---|---|---|---|"]
    for r in rows[:limit]:
        nm = r["Name"].replace("(anonymous namespace)::", "").replace("|", "\\|")
        nm = nm.split("(")[0] if "<" not in nm.split("(")[0] else nm.split("(")[0]
        out.append(f"| `{nm[:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
    return "\n".join(out)


def pmc(name: str, kernel_substr: str) -> dict:
    path = os.path.join(SRC, name, "run_counter_collection.csv")
    agg, n = collections.defaultdict(float), collections.defaultdict(int)
    for r in csv.DictReader(open(path)):
        if kernel_substr in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
    return {k: v / n[k] for k, v in agg.items()}


def last_json(log: str) -> list[dict]:
    out = []
    for line in open(os.path.join(SRC, log)):
        line = line.strip()
        if line.startswith("{"):
            try:
                out.append(json.loads(line))
            except json.JSONDecodeError:
                pass
    return out


def mega_lines() -> list[str]:
    """HBM-resident dataset runs (bench.py --device-data-gb), read from the committed jsonl lines."""
    out = []
    for name, label in (("bench_mega_data", "1M-sample steps streamed over the dataset"),
                        ("bench_mega_batch", "mega-batch: 256M samples per optimizer step"),
                        ("bench_wide_mega", "wide MLP 62->8192->8192->62, 1M-sample steps (16 x 64k micro-batches, "
                                            "gradient accumulation)")):
        path = os.path.join(DST, f"{name}.jsonl")
        if not os.path.exists(path):
            continue
        j = [json.loads(x) for x in open(path) if x.strip()][-1]
        g = dict(j.get("device_datagen") or j.get("datagen") or {})
        if "gib" not in g and g.get("draws"):
            g["gib"] = g["draws"] * 8 / 2 ** 30
        rate = f"**{j['value'] / 1e9:.2f} G samples/s**" if j["value"] > 1e8 else f"**{j['value'] / 1e6:.2f} M samples/s**"
        if "tflops_per_gpu" in j:
            rate += f" ({j['tflops_per_gpu']:.0f} TFLOP/s)"
        out.append(f"* {label}: {rate}, {j['ms_per_step']:.3f} ms/step, "
                   f"val acc {j.get('val', {}).get('acc', float('nan')):.4f}; dataset {g.get('gib', 0):.0f} GiB = "
                   f"{g.get('draws', 0) / 1e9:.1f} G draws generated on the GPU in {g.get('seconds', 0):.2f} s")
    if out:
        out = ["### HBM-resident dataset (`bench.py --device-data-gb 200`, draws generated on the GPU)", ""] + out + [""]
    return out


def main():
    os.makedirs(DST, exist_ok=True)
    for d in ("fused", "wide", "rf", "gbdt"):
        shutil.copy(os.path.join(SRC, d, "run_kernel_stats.csv"), os.path.join(DST, f"kernel_stats_{d}.csv"))
    for log in ("bench_headline", "bench_torch", "bench_wide", "gemm_bench", "rf_bench", "gbdt_bench",
                "bench_mega_data", "bench_mega_batch", "bench_wide_mega"):
        if not os.path.exists(os.path.join(SRC, f"{log}.log")):
            continue
        with open(os.path.join(DST, f"{log}.jsonl"), "w") as f:
            for j in last_json(f"{log}.log"):
                f.write(json.dumps(j) + "\n")
    f1 = pmc("fused_pmc", "mlp_fused_train")
    f2 = pmc("fused_pmc2", "mlp_fused_train")
    w = pmc("wide_pmc", "gemm256_pp16_kernel<1, 1, 0, 0") or pmc("wide_pmc", "gemm256_pp_kernel<1, 1, 0, 0>") or pmc("wide_pmc", "gemm256_nt_kernel<1, 1, 0, 0>")
    wcyc = w.get("GRBM_GUI_ACTIVE", 0) / 8.0
    w_busy = w.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, 1024 * wcyc) if wcyc else float("nan")
    head = last_json("bench_headline.log")[-1]
    torch_b = last_json("bench_torch.log")[-1]
    wide = last_json("bench_wide.log")[-1]
    waves = f1.get("SQ_WAVES", 1)
    cyc = f2.get("GRBM_GUI_ACTIVE", 0) / 8.0  # summed over 8 XCDs
    mfma_busy = f1.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, 1024 * cyc) if cyc else float("nan")
    lines = [
        "# Profiles (1x MI355X, rocprofv3; refreshed by `tools/collect_profiles.sh` + `tools/summarize_profiles.py`)",
        "",
        "## Headline: fused 62->128->62 MLP train step (1M samples / step)",
        "",
        f"* bench: **{head['value'] / 1e9:.2f} G samples/s**, {head['ms_per_step']:.4f} ms/step (hipGraph), "
        f"val acc {head['val'].get('acc', float('nan')):.4f} vs trivial {head['val'].get('trivial_acc', float('nan')):.4f}; "
        f"iid-data control: {head.get('val_iid', {}).get('hits_main', float('nan')):.3f} main hits (chance 0.5)",
        f"* same model, plain PyTorch eager (hipBLASLt GEMMs + torch Adam): {torch_b['value'] / 1e6:.0f} M samples/s "
        f"({head['value'] / torch_b['value']:.0f}x slower)",
        "",
        stats_table("fused", 6),
        "",
        "PMC (train kernel, per dispatch):",
        "",
        "| counter | value | reading |",
        "|---|---|---|",
        f"| SQ_WAVES | {waves:.0f} | 8 waves (2 units: 2 forward + 2 backward waves) x 256 CUs |",
        f"| SQ_INSTS_MFMA / wave | {f1.get('SQ_INSTS_MFMA', 0) / waves:.0f} | 32 per tile per forward wave, 26 per tile per backward wave |",
        f"| SQ_INSTS_VALU / wave | {f1.get('SQ_INSTS_VALU', 0) / waves:.0f} | |",
        f"| SQ_WAIT_ANY / SQ_WAVE_CYCLES | {f1.get('SQ_WAIT_ANY', 0) / max(1, f1.get('SQ_WAVE_CYCLES', 1)):.2f} | latency-bound share |",
        f"| SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES | {f1.get('SQ_ACTIVE_INST_VALU', 0) / max(1, f1.get('SQ_WAVE_CYCLES', 1)):.2f} | |",
        f"| MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / SIMD-cycles) | {mfma_busy:.2f} | |",
        f"| SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE | {f2.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, f2.get('SQ_LDS_IDX_ACTIVE', 1)):.2f} | |",
        "",
        *mega_lines(),
        "## Wide MLP 62->8192->8192->62 (64k samples / step)",
        "",
        f"* bench: {wide['value'] / 1e6:.2f} M samples/s, {wide['ms_per_step']:.1f} ms/step, "
        f"{wide.get('tflops_per_gpu', float('nan')):.0f} TFLOP/s effective",
        "",
        stats_table("wide", 12),
        "",
        f"256x256 ping-pong GEMM (8192^2 layer, per dispatch) PMC: MFMA busy {w_busy:.2f} of SIMD-cycles, "
        f"{w.get('SQ_INSTS_MFMA', 0):.3g} MFMA insts, FETCH_SIZE {w.get('FETCH_SIZE', 0) / 1024:.0f} MB",
        "",
        "GEMM micro-benchmark vs torch.matmul (hipBLASLt), same GPU: see `gemm_bench.jsonl`.",
        "",
        "## Random forest (100 trees, depth 8, 700k rows)",
        "",
        stats_table("rf", 6),
        "",
        "## GBDT (tools/gbdt_bench.py: reference config 500 rounds x 62 boosters on ~930 rows, then 50 rounds on 183k synthetic rows; depth 3)",
        "",
        stats_table("gbdt", 10),
        "",
        "Raw per-kernel stats: `kernel_stats_*.csv`; benchmark lines: `*.jsonl`.",
    ]
    with open(os.path.join(DST, "README.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"wrote {DST}/README.md")


def pmc_ab(root: str, kernel_substr: str = "mlp_fused_train") -> None:
    """Markdown table of the train kernel's PMC (median per dispatch) for every arm directory under
    root (tools/gpu_round.sh pmc-ab: <arm>/p1, <arm>/p2), with the derived utilisations."""
    import statistics

    rows = []
    for arm in sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))):
        vals = collections.defaultdict(list)
        for p in ("p1", "p2"):
            path = os.path.join(root, arm, p, "run_counter_collection.csv")
            if not os.path.exists(path):
                continue
            for r in csv.DictReader(open(path)):
                if kernel_substr in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if not vals:
            continue
        m = {k: statistics.median(v) for k, v in vals.items()}
        rows.append((arm, m))
    if not rows:
        print("no counter data under", root)
        return
    keys = sorted({k for _, m in rows for k in m})
    print("| counter | " + " | ".join(a for a, _ in rows) + " |")
    print("|---|" + "---|" * len(rows))
    for k in keys:
        print(f"| {k} | " + " | ".join(f"{m.get(k, float('nan')):.4g}" for _, m in rows) + " |")

    def der(m):
        g = m.get("GRBM_GUI_ACTIVE", float("nan")) / 8  # cycles per XCD
        wc = m.get("SQ_WAVE_CYCLES", float("nan"))
        return {
            "MFMA busy (of 1024 SIMDs)": m.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / 1024 / g,
            "LDS active (IDX_ACTIVE / 256 CUs / cycles)": m.get("SQ_LDS_IDX_ACTIVE", float("nan")) * 4 / 256 / g,
            "LDS bank conflict / IDX_ACTIVE": m.get("SQ_LDS_BANK_CONFLICT", float("nan")) / m.get("SQ_LDS_IDX_ACTIVE", float("nan")),
            "VALU active / wave-cycles": m.get("SQ_ACTIVE_INST_VALU", float("nan")) / wc,
            "LDS issue-wait / wave-cycles": m.get("SQ_WAIT_INST_LDS", float("nan")) / wc,
            "WAIT_INST_ANY / wave-cycles": m.get("SQ_WAIT_INST_ANY", float("nan")) / wc,
            "WAIT_ANY / wave-cycles": m.get("SQ_WAIT_ANY", float("nan")) / wc,
            "kernel cycles per XCD": g,
        }
    print()
    print("| derived | " + " | ".join(a for a, _ in rows) + " |")
    print("|---|" + "---|" * len(rows))
    ds = [der(m) for _, m in rows]
    for k in ds[0]:
        print(f"| {k} | " + " | ".join(f"{d[k]:.3f}" if d[k] < 100 else f"{d[k]:.4g}" for d in ds) + " |")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pmc-ab":
    pmc_ab(sys.argv[2])
    sys.exit(0)

if __name__ == "__main__":
    main()
