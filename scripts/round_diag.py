import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import imsame_amd
from tests import synth
ref, rst = synth.make_reference_arr(50_000_000, 2_000, seed=42)
q, qs = synth.make_reads_arr(ref, 1_000_000, 150, seed=43)
d = imsame_amd.Device(0)
d.index(ref, rst); d.set_query(q, qs)
for _ in range(2):
    res, _, st = d.align(n_threads=16)
    print("ms_seed", st.ms_seed, "ms_nw", st.ms_nw, "total", st.ms_total, "rounds", st.rounds, flush=True)
