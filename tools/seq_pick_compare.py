"""Reservoir vs inverse-CDF pick in the sequential chain (oracle, chunk = 1), 200 seeds each on C1 (T = 1000):
means and standard errors of [maxlik purity, maxlik ARI, maxlik K, last ARI, last K].  CPU, ~2 min on 7 cores.
usage: python tools/seq_pick_compare.py"""
import sys, json, numpy as np
sys.path.insert(0,'tests/golden'); sys.path.insert(0,'oracle'); sys.path.insert(0,'.')
import make_chain_stats as M
from multiprocessing import Pool
def f(a):
    s, pick = a
    r = M.run(s, chunk=1, pick=pick)
    return [r['maxlik']['purity'], r['maxlik']['ari'], r['maxlik']['K'], r['last']['ari'], r['last']['K']]
if __name__ == '__main__':
    with Pool(7) as p:
        inv = np.array(p.map(f, [(100000+s, 'invcdf') for s in range(200)]))
        res = np.array(p.map(f, [(200000+s, 'reservoir') for s in range(200)]))
    for n,a in (('invcdf',inv),('reservoir',res)):
        print(n, np.nanmean(a,0).round(4), (np.nanstd(a,0)/np.sqrt(len(a))).round(4))
    json.dump({'invcdf': inv.tolist(), 'reservoir': res.tolist()}, open('gpurun_out/seq_pick_compare.json','w'))
