"""Write tests/golden/figure1.json: the reference's Figure-1 DAG fixture and its known answers.

Data transcribed from the reference test (xenowits/dag-rider):
  DAG            process/process_internal_test.go:86-283 (createDag): rounds 0..4, each
                 with 5 slots; slot 0 keeps the zero vertex {0,0} (:89-100), slots 1..4
                 are sources 1..4; edges :103-280.
  TestPath       process/process_internal_test.go:20-83, with n=5 slots, f=1 (:9-14).
Derived answers (hand-derived from process.go semantics, Go-unexecuted):
  waveReady(1), orderVertices with single-leader stacks, strong reach set of (4,1).
The all-pairs path matrices are produced by the literal C restatement
(oracle/ref_literal.c) and are regression vectors, not reference outputs.

Run: python tests/golden/make_figure1.py   (needs `make oracle`)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

# (round, source) -> (strong targets, weak targets); process_internal_test.go:103-280
EDGES = {
    (1, 1): ([(0, 1), (0, 2), (0, 3)], []),
    (1, 2): ([(0, 1), (0, 2), (0, 3)], []),
    (1, 3): ([(0, 1), (0, 2), (0, 3)], []),
    (1, 4): ([(0, 1), (0, 2), (0, 3)], []),
    (2, 1): ([(1, 1), (1, 2), (1, 4)], []),
    (2, 2): ([(1, 1), (1, 2), (1, 4)], []),
    (2, 3): ([(1, 1), (1, 3), (1, 4)], []),
    (2, 4): ([(1, 1), (1, 2), (1, 4)], []),
    (3, 1): ([(2, 1), (2, 3)], []),
    (3, 2): ([(2, 1), (2, 2), (2, 3)], []),
    (3, 3): ([(2, 1), (2, 2), (2, 3)], []),
    (4, 1): ([(3, 1), (3, 2), (3, 3)], [(2, 4)]),
}


def build():
    rounds = []
    for r in range(5):
        slots = [{"id": [0, 0], "strong": [], "weak": []}]  # ghost slot 0
        for s in range(1, 5):
            st, wk = EDGES.get((r, s), ([], []))
            slots.append({"id": [r, s], "strong": [list(e) for e in st], "weak": [list(e) for e in wk]})
        rounds.append(slots)
    return rounds


def main():
    from dag_rider_amd.dag import Vertex, VertexID, flatten_lists
    import oracle

    rounds = build()
    dag = [[Vertex(VertexID(*v["id"]), b"", [VertexID(*e) for e in v["strong"]],
                   [VertexID(*e) for e in v["weak"]]) for v in rnd] for rnd in rounds]
    ld = oracle.LDag(arrays=flatten_lists(dag))
    ids = [(r, s) for r in range(5) for s in range(0, 5)]
    allpairs = {}
    for strong in (True, False):
        allpairs["strong" if strong else "any"] = [[ld.path(a, b, strong) for b in ids] for a in ids]
    out = {
        "source": "xenowits/dag-rider process/process_internal_test.go:86-283 (createDag)",
        "n": 4,
        "faulty": 1,
        "rounds": rounds,
        "test_path": [  # reference-authored known answers, process_internal_test.go:20-83
            {"from": [3, 1], "to": [2, 3], "strong": True, "want": True, "ref": "process_internal_test.go:20-31"},
            {"from": [3, 3], "to": [1, 4], "strong": True, "want": True, "ref": "process_internal_test.go:33-44"},
            {"from": [4, 1], "to": [2, 4], "strong": False, "want": True, "ref": "process_internal_test.go:46-57"},
            {"from": [4, 1], "to": [1, 1], "strong": False, "want": True, "ref": "process_internal_test.go:59-70"},
            {"from": [3, 3], "to": [2, 4], "strong": False, "want": False, "ref": "process_internal_test.go:72-83"},
        ],
        "derived": {  # SURVEY.md s4, derived from process.go, Go-unexecuted
            "wave_ready_1": {"leader": [1, 1], "voters": [False, True, False, False, False], "vcount": 1,
                             "commit": False},
            "order_vertices": [
                {"stack": [[4, 1]], "p_round": 4,
                 "want": [[1, 1], [1, 2], [1, 3], [1, 4], [2, 1], [2, 2], [2, 3], [2, 4], [3, 1], [3, 2], [3, 3],
                          [4, 1]]},
                {"stack": [[3, 3]], "p_round": 4,
                 "want": [[1, 1], [1, 2], [1, 3], [1, 4], [2, 1], [2, 2], [2, 3], [3, 3]]},
                {"stack": [[1, 1]], "p_round": 4, "want": [[1, 1]]},
            ],
            "strong_reach_4_1": [[0, 1], [0, 2], [0, 3], [1, 1], [1, 2], [1, 3], [1, 4], [2, 1], [2, 2], [2, 3],
                                 [3, 1], [3, 2], [3, 3], [4, 1]],
        },
        "allpairs_ids": ids,
        "allpairs": allpairs,
        "allpairs_source": "oracle/ref_literal.c (literal restatement of process.go:89-148)",
    }
    with open(os.path.join(HERE, "figure1.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote figure1.json")


if __name__ == "__main__":
    main()
