"""Compact table of a tools/variant_bench.py log: ms per launch per scene and
variant (fwd = sample-buffer forward, render = fused/two-kernel render, adj =
bounded adjoint, adju / renderu = unbounded, *8 = a 1/8 interleaved share,
band = a 64-row band), plus any correctness line that is not exact."""
import ast
import sys

KEYS = ("fwd_ms", "render_ms", "adj_ms", "adj5_ms", "adju_ms", "renderu_ms", "render8_ms", "adj8_ms", "band_ms")
for line in open(sys.argv[1]):
    if "MISMATCH" in line:
        print(line.rstrip())
    if "_ms" not in line or line.startswith("{"):
        continue
    sc, v, d = line.split(" ", 2)
    d = ast.literal_eval(d.strip().replace("np.float64(", "(").replace(")", ")"))
    print("%-9s %-9s" % (sc, v), " ".join("%s=%.4f" % (k[:-3], d[k]) for k in KEYS if k in d))
