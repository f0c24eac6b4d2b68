import sys, time
sys.path.insert(0, '/root/repo')
import panman_amd
t=time.time(); off, idx, root = panman_amd.random_join_tree(8_000_000, seed=1); print('gen', round(time.time()-t,2), flush=True)
eng = panman_amd.Engine(0)
t=time.time(); eng.tree_upload(off, idx, root); print('upload', round(time.time()-t,2), flush=True)
t=time.time(); eng.synth_columns(0, 3750, seed=2); print('synth', round(time.time()-t,2), flush=True)
import resource; print('maxrss GB', resource.getrusage(resource.RUSAGE_SELF).ru_maxrss/1e6)
