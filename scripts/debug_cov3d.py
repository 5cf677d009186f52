import sys, os
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [R, os.path.join(R, "generalized-icp_amd"), os.path.join(R, "tests")]
import numpy as np
import gicp
from gicp import synthetic as S
from oracle import gicp_oracle as O
src, tgt, Tgt = S.scene_pair_3d(int(sys.argv[1]) if len(sys.argv) > 1 else 20000)
eng = gicp.Engine(0)
p = gicp.default_params(3, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
eng.set_target(tgt, p)
cg = eng.neighbor_counts("target"); Cg = eng.covariances("target")
idx, valid, dist = O.neighbourhoods(tgt, 1.0, 21)
co = np.minimum(valid.sum(1), 20)
bad = np.nonzero(cg != co)[0]
print("count mismatches", len(bad), "of", len(tgt))
for i in bad[:10]:
    print(i, "gpu", cg[i], "oracle", co[i], "d20..21", dist[i, 18:21])
C_or, _ = O.covariances(tgt, 1.0)
err = np.max(np.abs(Cg - C_or), axis=(1, 2))
print("cov err quantiles", np.quantile(err, [0.5, 0.99, 0.999, 1.0]), "n>1e-6", np.sum(err > 1e-6))
w = np.argsort(err)[-5:]
for i in w:
    ev = np.linalg.eigvalsh(np.cov(tgt[idx[i][valid[i]][:20]].T))
    print(i, err[i], "cnt", cg[i], co[i], "eig", ev)
