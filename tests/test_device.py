"""sfl_amd.device (the slice of secretflow.device the aggregator touches):
device objects nested in call arguments resolve to their values, whatever
container holds them (namedtuples and other tuple subclasses)."""
import collections

import numpy as np
import pytest

from sfl_amd import device as D

Pair = collections.namedtuple("Pair", "a b")


class Tagged(list):
    pass


def test_nested_arguments_resolve_in_any_container():
    alice = D.PYU("alice", gpu=None)
    x = D.PYUObject(alice, np.arange(3))
    seen = {}

    def fn(p, q, t, d, plain):
        seen.update(p=p, q=q, t=t, d=d, plain=plain)
        return 0

    alice(fn)(Pair(x, 5), Pair(1, 2), Tagged([x, 7]), {"k": [x]}, (x,))
    assert isinstance(seen["p"], Pair) and np.array_equal(seen["p"].a, np.arange(3)) and seen["p"].b == 5
    assert seen["q"] == Pair(1, 2)
    assert type(seen["t"]) is Tagged and np.array_equal(seen["t"][0], np.arange(3)) and seen["t"][1] == 7
    assert np.array_equal(seen["d"]["k"][0], np.arange(3))
    assert type(seen["plain"]) is tuple


def test_unchanged_containers_pass_through():
    alice = D.PYU("alice", gpu=None)
    p = Pair(1, 2)
    got = []
    alice(lambda v: got.append(v))(p)
    assert got[0] is p


def test_foreign_object_is_refused():
    alice, bob = D.PYU("alice", gpu=None), D.PYU("bob", gpu=None)
    with pytest.raises(ValueError, match="move it with .to"):
        alice(lambda v: v)(Pair(D.PYUObject(bob, 1), 2))
