"""Study of rl-results.csv seq_hc at alpha .25, gamma .95 (tests/test_gpu_gamma.py allowance;
DESIGN.md §2.1): 16,384 oracle gym episodes (42 defenders, 2048 steps, SM1) and 2,048 honest,
the distribution of a 100-episode mean by bootstrap, and the z of the reference value.
Output: profiles/r03_rl_point_study.log"""
import sys, time, numpy as np
import os; R = os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."); sys.path.insert(0, os.path.join(R, "tests")); sys.path.insert(0, R)
import oracle_py as O
from cpr_amd import device, _lib as L
t0=time.time()
res={}
for name,pid in (("sm1",L.POLICY_SAPIRSHTEIN_2016_SM1),("honest",L.POLICY_HONEST)):
    cfg,_=device.make_config(alpha=0.25,gamma=0.95,defenders=42,policy=pid,max_steps=2048,seed=0x7A11)
    n = 16384 if name=="sm1" else 2048
    rec=O.run_episodes(cfg,0,n,threads=8)
    res[name]=rec["reward_attacker"]/rec["progress"]
    print(name, n, res[name].mean(), res[name].std(ddof=1), time.time()-t0, flush=True)
x=res["sm1"]; ref=0.3036808105715036
m=x.mean(); sd=x.std(ddof=1)
from scipy import stats
print("skew", stats.skew(x), "kurt", stats.kurtosis(x))
rng=np.random.default_rng(1)
B=200000
means=x[rng.integers(0,len(x),size=(B,100))].mean(axis=1)
print("bootstrap P(mean100 >= ref) =", (means>=ref).mean(), " normal approx:", 1-stats.norm.cdf((ref-m)/(sd/10)))
print("z(ref vs 100-mean, se from sample)", (ref-m)/np.sqrt(sd**2/100+sd**2/len(x)))
