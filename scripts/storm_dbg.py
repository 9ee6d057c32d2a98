import sys
sys.path[:0] = ["/root/repo/raft-simulation_amd", "/root/repo/tests", "/root/repo/oracle"]
import numpy as np
import helpers
cfg = dict(n_clusters=2048, nodes=5, seed=1, log_cap=1024, client_ppm=80000, client_period=16384,
           client_burst=2048, client_redirects=4, drop_ppm=100000, dup_ppm=10000, dmin=1, dmax=50,
           part_ppm=100000, variant_flags=int(sys.argv[1]))
g, r = helpers.gpu(**cfg), helpers.oracle(**cfg)
for i in range(8):
    g.step(1000); r.step(1000)
    bad = np.nonzero(g.digest() != r.digest())[0]
    print("chunk", i, "launches", g.last_step_timing()[1], "bad", len(bad), flush=True)
    if len(bad):
        c = int(bad[0])
        print(helpers.describe_cluster_diff(g, r, c))
        break
print(g.counters() == r.counters())
