"""Write tests/golden/large_replay.json.gz: full-size golden vectors for C3, C4 and C5.

C3 (n=256 x 10k rounds, weak-heavy) and C4 (n=1024 x 4k rounds): the complete
replay outputs (commit bits, vote counts, pushed leaders, per-pop count / digest /
edges, edge totals) in DR_CHAIN_PERSISTENT with DR_DELIVER_REF and with
DR_DELIVER_PAPER; and DR_CHAIN_LITERAL with DR_DELIVER_REF (the reference's Q1
behaviour: every commit chains down to wave 1, O(w^2) pops) as a replay fingerprint
plus push count and edge totals.  C5 (4096 independent n=128 x 128-round DAGs, seeds 5000+i):
one replay fingerprint per DAG (tests/dagutil.replay_fingerprint) for
PERSISTENT/REF, and for the first 64 DAGs also LITERAL/REF and PERSISTENT/PAPER.

Each config also records the generator fingerprint (dagutil.dag_fingerprint) so a
drifting generator is caught before any replay is compared.

Produced by the bitset restatement (oracle/ref_bitset.c).  The literal restatement
(oracle/ref_literal.c, the reference algorithm line by line) is run on a prefix of
every config first and must agree: 8 waves of C3, 4 of C4 (all threads), 4 of each
of the first 64 C5 DAGs.  Regression vectors: the reference (Go) cannot
run in this image, so these are not reference outputs.
Run: python tests/golden/make_large.py [--c34]   (--c34: redo C3/C4 only and keep
the committed C5 rows; about 10 minutes on 8 cores)
"""
import gzip
import json
import multiprocessing
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

C5_COUNT = 4096
C5_DETAIL = 64
C5_LITERAL_WAVES = 4


def replay_dict(r):
    return dict(commit="".join(str(int(x)) for x in r.commit), vcount=r.vcount.tolist(),
                push_off=r.push_off.tolist(), push_wave=r.push_wave.tolist(),
                pop_count=[str(x) for x in r.pop_count], pop_digest=[str(x) for x in r.pop_digest],
                pop_edges=[str(x) for x in r.pop_edges], commit_edges=str(r.commit_edges),
                chain_edges=str(r.chain_edges), deliver_edges=str(r.deliver_edges))


def literal_prefix_check(cfg, d, r, k, nthreads=1):
    """The literal restatement on waves 1..k must match the bitset replay's prefix."""
    import oracle

    lit = oracle.LDag(packed=d, nrounds=4 * k + 1).replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT,
                                                            oracle.DELIVER_REF, nthreads=nthreads)
    npop = int(lit.push_off[k])
    assert lit.commit.tolist() == r.commit[:k].tolist()
    assert lit.vcount.tolist() == r.vcount[:k].tolist()
    assert lit.pop_digest.tolist() == r.pop_digest[:npop].tolist()
    assert lit.pop_count.tolist() == r.pop_count[:npop].tolist()


def c5_one(i):
    import oracle
    from dag_rider_amd import gen
    from dagutil import dag_fingerprint, replay_fingerprint

    cfg = gen.c5_config(i)
    d = gen.generate(cfg)
    bs = oracle.PDag(d)
    r = bs.replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF, nthreads=1)
    row = dict(dag=dag_fingerprint(d), persistent_ref=replay_fingerprint(r))
    if i < C5_DETAIL:
        literal_prefix_check(cfg, d, r, C5_LITERAL_WAVES)
        for key, cm, dm in (("literal_ref", oracle.CHAIN_LITERAL, oracle.DELIVER_REF),
                            ("persistent_paper", oracle.CHAIN_PERSISTENT, oracle.DELIVER_PAPER)):
            row[key] = replay_fingerprint(bs.replay(cfg.faulty, cfg.nwaves, cm, dm, nthreads=1))
    return row


def main():
    import oracle
    from dag_rider_amd import gen
    from dagutil import dag_fingerprint, replay_fingerprint

    out = {}
    for name, k in (("c3", 8), ("c4", 4)):
        cfg = gen.CONFIGS[name]
        t0 = time.time()
        d = gen.generate(cfg, nthreads=8)
        bs = oracle.PDag(d)
        ent = dict(config=cfg.__dict__, dag=dag_fingerprint(d))
        for key, dm in (("persistent_ref", oracle.DELIVER_REF), ("persistent_paper", oracle.DELIVER_PAPER)):
            r = bs.replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, dm, nthreads=8)
            assert r.rc == 0
            if dm == oracle.DELIVER_REF:
                literal_prefix_check(cfg, d, r, k, nthreads=8)
            ent[key] = replay_dict(r)
        ent["literal_prefix_waves"] = k
        r = bs.replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_LITERAL, oracle.DELIVER_REF, nthreads=8)
        assert r.rc == 0
        ent["literal_ref"] = dict(fingerprint=replay_fingerprint(r), n_push=int(len(r.push_wave)),
                                  commit_edges=str(r.commit_edges), chain_edges=str(r.chain_edges),
                                  deliver_edges=str(r.deliver_edges))
        out[name] = ent
        print(f"{name}: {time.time() - t0:.1f} s", flush=True)
    if "--c34" in sys.argv:
        from dagutil import load_large

        out["c5"] = load_large()["c5"]
        with gzip.open(os.path.join(HERE, "large_replay.json.gz"), "wt") as f:
            json.dump(out, f)
        print("wrote large_replay.json.gz (C5 rows kept)")
        return

    t0 = time.time()
    base = gen.CONFIGS["c5"]
    c5 = dict(config=base.__dict__, count=C5_COUNT, literal_prefix_waves=C5_LITERAL_WAVES)
    with multiprocessing.get_context("spawn").Pool(8) as pool:  # the parent already ran OpenMP: no fork
        rows = pool.map(c5_one, range(C5_COUNT), chunksize=16)
    for key in ("dag", "persistent_ref", "literal_ref", "persistent_paper"):
        c5[key] = [x[key] for x in rows if key in x]
    out["c5"] = c5
    print(f"c5: {time.time() - t0:.1f} s", flush=True)
    with gzip.open(os.path.join(HERE, "large_replay.json.gz"), "wt") as f:
        json.dump(out, f)
    print("wrote large_replay.json.gz")


if __name__ == "__main__":
    main()
