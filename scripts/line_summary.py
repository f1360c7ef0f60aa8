#!/usr/bin/env python3
"""Print the key numbers of bench.py JSON lines (tooling)."""
import json
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        line = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    r = line["roofline"]
    cold = r.get("cold")
    print(f"{path}: value {line['value']} GiB/s, kernel {r['kernel_ms'] * 1000:.1f} us, frac {r['frac']}, "
          f"ceiling {r.get('read_ceiling_gbs')} GB/s, frac_of_ceiling {r.get('frac_of_ceiling')}"
          + (f"  (cold {cold['kernel_ms'] * 1000:.1f} us, frac {cold['frac']})" if cold else ""))
    for k in ("shard_2m", "mtu_1392", "ragged_g2", "large_64k", "frag_64k"):
        if k in line:
            p = line[k]
            cold = p.get("cold", {}).get("kernel_ms")
            print(f"  {k:10s} kernel {p['kernel_ms'] * 1000:7.1f} us  frac {p['frac']:.4f}  "
                  f"ceiling {p.get('read_ceiling_gbs')}  frac_of_ceiling {p.get('frac_of_ceiling')}"
                  + (f"  (cold {cold * 1000:.1f} us)" if cold else ""))
    v = line.get("verify_256")
    if v:
        print(f"  verify_256: host {v['host_us']} us + slot adjust {v['slot_adjust_us']} us, ring {v['ring_us']} us, "
              f"protocol {v['protocol_verify_received_us']} us, cpu 1 core {v['cpu_1core_us']} us, "
              f"crossover batch {v['crossover_batch']}")
        for b, row in v["sweep"].items():
            print(f"    batch {b:>6s}: host {row['host_us']:8.1f} us  cpu {row['cpu_1core_us']:8.1f} us")
