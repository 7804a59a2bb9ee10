import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import oracle as O
from noparama_amd import NealAlgorithm8, datasets
X = datasets.config_c3(N=30000)[0]
kw = dict(seed=91, kcap=1024)
a = NealAlgorithm8(8, device=0, **kw); b = NealAlgorithm8(8, device=0, **kw); o = O.Chain(8, **kw)
for c in (a, o): c.set_data(X); c.init_random(20)
a.sweep(7); o.sweep(7)
print("a==o after 7", np.array_equal(a.state()["z"], o.state()["z"]))
ck = a.checkpoint()
b.set_data(X); b.restore(ck)
sa, sb = a.state(), b.state()
print("restored equal:", sa["K"], sb["K"], np.array_equal(sa["z"], sb["z"]), np.array_equal(sa["mu"], sb["mu"]))
print("stats a", {k: a.stats()[k] for k in ("epoch","K","new_clusters")}, "b", {k: b.stats()[k] for k in ("epoch","K","new_clusters")})
for t in range(6):
    a.sweep(1); b.sweep(1); o.sweep(1)
    za, zb, zo = a.state()["z"], b.state()["z"], o.state()["z"]
    print(t, a.K, b.K, o.K, np.array_equal(za, zo), np.array_equal(zb, zo), (za != zb).sum())
