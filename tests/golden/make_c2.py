"""Write tests/golden/c2_replay.json: C2 (n=64 x 1000 rounds, seed 2) full replay outputs.

Produced by the bitset restatement (oracle/ref_bitset.c), after checking that the
literal restatement (oracle/ref_literal.c) agrees on the first `literal_prefix_waves`
waves.  Regression vectors: the reference (Go) cannot run here, so these are not
reference outputs.  Run: python tests/golden/make_c2.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import oracle
    from dag_rider_amd.gen import CONFIGS, generate

    cfg = CONFIGS["c2"]
    d = generate(cfg)
    r = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
    k = 6
    lit = oracle.LDag(packed=d, nrounds=4 * k + 1).replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
    npop = int(lit.push_off[k])
    assert lit.pop_digest.tolist() == r.pop_digest[:npop].tolist()
    out = dict(config=cfg.__dict__, commit=r.commit.tolist(), vcount=r.vcount.tolist(),
               push_wave=r.push_wave.tolist(), pop_count=[str(x) for x in r.pop_count],
               pop_digest=[str(x) for x in r.pop_digest], pop_edges=[str(x) for x in r.pop_edges],
               commit_edges=str(r.commit_edges), chain_edges=str(r.chain_edges), deliver_edges=str(r.deliver_edges),
               literal_prefix_waves=k)
    with open(os.path.join(HERE, "c2_replay.json"), "w") as f:
        json.dump(out, f)
    print("wrote c2_replay.json", int(r.commit.sum()), "commits")


if __name__ == "__main__":
    main()
