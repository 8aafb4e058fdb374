"""One line per bench.py JSON file: the headline and every secondary leg it carries (no GPU)."""
import json
import sys


def main() -> None:
    for path in sys.argv[1:]:
        for line in open(path):
            line = line.strip()
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            parts = [f"{path}: {d['value'] / 1e6:.1f} M votes/s", f"{d['ms_per_step']:.3f} ms/step", f"N={d['n_gpus']}"]
            rf = d.get("roofline", {})
            if rf.get("kernel_ms_avg"):
                parts.append(f"rec {rf['kernel_ms_avg']:.3f} ms frac {rf['frac']:.3f}")
            if "legs" in d:  # the compact line (round 6 on): one number per leg, failures in leg_errors
                for k, v in d["legs"].items():
                    parts.append(f"{k} {v / 1e6:.1f} M")
                for k, e in d.get("leg_errors", {}).items():
                    parts.append(f"{k} error: {e}")
            for k in ("wire", "end_to_end", "end_to_end_pinned", "end_to_end_concurrent", "stream", "config3", "config5"):
                if k in d and "legs" not in d:
                    v = d[k].get("value")
                    parts.append(f"{k} {v / 1e6:.1f} M" if v is not None else f"{k} error: {d[k].get('error')}")
            if "cpu_baseline" in d:
                c = d["cpu_baseline"]
                parts.append(f"cpu {c['value'] / 1e3:.1f} k" if "value" in c else f"cpu error: {c.get('error')}")
            elif "cpu_baseline" in d.get("leg_errors", {}):
                parts.append(f"cpu error: {d['leg_errors']['cpu_baseline']}")
            if "gathered_results" in d:
                parts.append(f"gathered {d['gathered_results']}")
            if "counters_per_step" in d:
                parts.append(f"verified {d['counters_per_step']['verified_votes']}")
            print(", ".join(parts))


if __name__ == "__main__":
    main()
