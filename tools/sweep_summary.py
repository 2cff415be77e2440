#!/usr/bin/env python3
"""Summarise a c5 sweep (tools/sweep.py JSON lines): bit-exact count, device-resident HBM
fractions and host-path rates, medians overall and by chunk size.

python tools/sweep_summary.py profiles/r01_v33_sweep_c5.jsonl
"""
import json
import statistics as st
import sys


def main():
    rows = [r for r in (json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")) if "method" in r]
    print(f"points {len(rows)}, bit-exact {sum(r['bit_exact'] for r in rows)}")
    med = lambda key, rs: st.median(r[key] for r in rs)  # noqa: E731
    print(f"device encode frac median {med('enc_hbm_frac', rows):.3f} (min {min(r['enc_hbm_frac'] for r in rows):.3f}), "
          f"decode {med('dec_hbm_frac', rows):.3f} (min {min(r['dec_hbm_frac'] for r in rows):.3f})")
    for C in sorted({r["chunk"] for r in rows}):
        rs = [r for r in rows if r["chunk"] == C]
        print(f"C={C >> 10:5d} KiB  device enc {med('enc_hbm_frac', rs):.3f} dec {med('dec_hbm_frac', rs):.3f}  "
              f"host enc {med('host_enc_gibps', rs):5.1f} dec {med('host_dec_gibps', rs):5.1f} GiB/s")
    if "enc_h2d_link_frac" in rows[0]:
        for key in ("enc_h2d_link_frac", "dec_h2d_link_frac"):
            lo = sorted(rows, key=lambda r: r[key])[:3]
            print(f"host {key} median {med(key, rows):.3f}, lowest " +
                  ", ".join(f"{r['method'][:2]}({r['k']}+{r['m']}) {r['chunk'] >> 10} KiB {r[key]:.3f}" for r in lo))


if __name__ == "__main__":
    main()
