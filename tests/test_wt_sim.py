"""K1's wavelet-tree layout and descents restated on the host (tools/wt_sim.py) against per-event decisions, for
every rank-block width the plan can take (32, 64 and 128 ranks). A design check of replayable_wt.hip, CPU only."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))

import wt_sim  # noqa: E402


def test_wt_sim_block_widths():
    rng = random.Random(11)
    for bb in (5, 6, 7):
        for n in (9, 31, 64, 65, 127, 128, 129, 300, 1030):
            for m in (3, 1000, (1 << 31) + 5, (1 << 32) - 1):
                cm = [rng.randrange(m) for _ in range(n)]
                e = rng.sample(range(4096), n)
                img = wt_sim.build(cm, e, [0] * n, bb=bb)
                for _ in range(8):
                    d = rng.choice([0, n, rng.randrange(n + 1)])
                    Hm, Hm2 = rng.randrange(m), rng.randrange(m)
                    RA = sum(1 for x in cm if x < m - Hm)
                    RB = sum(1 for x in cm if x < m - Hm2)
                    bW, bk = wt_sim.brute(cm, e, d, Hm, Hm2, m)
                    # the kernel's descents, and the count-guided alternative measured and rejected in round 5
                    for q in (wt_sim.query, wt_sim.query_quantile):
                        W, kA, kB = q(img, d, RA, RB, Hm, Hm2, m)
                        assert W == bW
                        assert max(x for x in (kA, kB) if x is not None) == bk
