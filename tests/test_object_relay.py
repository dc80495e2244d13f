"""The object-level relay simulator (oracle/object_relay.py, bench.py's 1-core CPU baseline
leg) reproduces the reference-harness fixtures: first-receipt round, lowest-id sender and
per-round relay counts, for flood, gossip and churn."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden, trim_zeros
from oracle.object_relay import ObjectRelay


@pytest.mark.parametrize("name", golden_cases())
def test_object_relay_matches_reference_harness(name):
    z = load_golden(name)
    sim = ObjectRelay(z["rowptr"], z["colidx"], str(z["mode"]), int(z["fanout"]), int(z["gossip_seed"]),
                      int(z["churn_threshold"]), int(z["churn_seed"]))
    relays = sim.run(z["src"])
    hop, par = sim.planes(len(z["rowptr"]) - 1, len(z["src"]))
    np.testing.assert_array_equal(hop, z["hop"])
    np.testing.assert_array_equal(par, z["parent"])
    np.testing.assert_array_equal(trim_zeros(relays), trim_zeros(z["round_relays"]))


def test_object_relay_bounded_sample_stops_early():
    z = load_golden("c2_rrg1000_flood")
    sim = ObjectRelay(z["rowptr"], z["colidx"])
    relays = sim.run(z["src"][:1], max_relays=500)
    assert 500 <= sum(relays) < 8 + 999 * 7
