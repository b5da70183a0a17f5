"""Writes tests/golden/figure1.drw1: the Figure-1 DAG (process_internal_test.go:86-283,
tests/golden/figure1.json) with a block on slot 1 of round 2, as dag_rider_amd/wire.py
encodes it.  go/dagridergpu/wire/wire_test.go decodes and re-encodes these bytes;
tests/test_wire.py checks wire.py still writes them.

usage: python tests/golden/make_wire_fixture.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from dag_rider_amd import wire  # noqa: E402
from dagutil import figure1  # noqa: E402


def fixture_dag():
    _, dag = figure1()
    dag[2][1].block = b"tx-batch"
    return dag


if __name__ == "__main__":
    with open(os.path.join(HERE, "figure1.drw1"), "wb") as f:
        f.write(wire.encode(fixture_dag()))
