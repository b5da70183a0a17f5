"""Probe: does the replay graph capture succeed with / without torch initialised first?"""
import sys

if sys.argv[1] == "torch":
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine, Replayer
from dag_rider_amd.gen import CONFIGS, generate

cfg = CONFIGS[sys.argv[2]]
d = generate(cfg, nthreads=16)
e = Engine(cfg.n, cfg.faulty, d.nrounds, 0)
e.append_packed(d)
if sys.argv[3] == "replayer":
    step = Replayer(e, cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    e.set_phase_timing(1)
    for i in range(4):
        step()
        print(sys.argv[1:], i, e.replay_graph_state(), step.ms_summary, flush=True)
else:
    e.set_phase_timing(1)
    for i in range(4):
        r = e.replay(cfg.nwaves)
        print(sys.argv[1:], i, e.replay_graph_state(), r.ms["summary"], flush=True)
