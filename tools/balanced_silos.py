"""Find generations g_k for silos 10.0.0.{k+1}:11111 whose consistent hashes
(SiloAddress.GetConsistentHashCode, SiloAddress.cs:164-173) sit near
-2^31 + k * 2^32 / S, so that the LocalGrainDirectory ring (one point per silo,
LocalGrainDirectory.cs:477-545) gives every silo ~1/S of the hash space.

Orleans allocates a generation as seconds since 2010 (SiloAddress.cs:72-76), so
any positive int is a legitimate generation; only the membership snapshot changes,
never the routing rule.  Prints the generation list bench.py hard-codes.

usage: python tools/balanced_silos.py [S] [max_gen]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from orleans_amd import graindispatch as g  # noqa: E402


def main():
    s = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    max_gen = int(sys.argv[2]) if len(sys.argv) > 2 else 300000
    gens = []
    for k in range(s):
        target = -(1 << 31) + k * (1 << 32) // s
        best = None
        for gen in range(1, max_gen):
            h = g.silo_consistent_hash(f"10.0.0.{k + 1}", 11111, gen)
            d = abs(h - target)
            if best is None or d < best[0]:
                best = (d, gen, h)
        gens.append(best[1])
        print(f"silo 10.0.0.{k + 1}:11111 gen {best[1]} hash {best[2]} (target {target}, off {best[0]})", flush=True)
    print("GENS =", gens)


if __name__ == "__main__":
    main()
