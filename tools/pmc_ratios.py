"""Derived per-kernel ratios from tools/summarize_pmc.py output (stdin)."""
import sys

cur, d = None, {}
for line in sys.stdin:
    if not line.startswith(" "):
        cur = line.strip()
        d[cur] = {}
        continue
    p = line.split()
    d[cur][p[0]] = float(p[2].split("=")[1])
for k, c in d.items():
    if not k.startswith("k_") or "SQ_WAVES" not in c:
        continue
    g = lambda n: c.get(n, float("nan"))
    print(f"{k:18s} lane_util={g('SQ_THREAD_CYCLES_VALU') / g('SQ_ACTIVE_INST_VALU') / 64:.2f} "
          f"wait={g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.2f} active={g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.2f} "
          f"valu/wave={g('SQ_INSTS_VALU') / g('SQ_WAVES'):.0f} salu/wave={g('SQ_INSTS_SALU') / g('SQ_WAVES'):.0f} "
          f"vmem/wave={g('SQ_INSTS_VMEM_RD') / g('SQ_WAVES'):.0f} smem/wave={g('SQ_INSTS_SMEM') / g('SQ_WAVES'):.0f} "
          f"lds/wave={g('SQ_INSTS_LDS') / g('SQ_WAVES'):.0f} "
          f"l2hit={g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.2f} waves={g('SQ_WAVES'):.3g}")
