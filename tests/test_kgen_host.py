"""The K_gen interpreter body (siddhi_amd/csrc/kgen.h), compiled for the host, against the CPU oracle
on every reference KAT stream (bit-exact match tuples, same delivery order) and on the KATs' expected
rows. This pins the device kernel's per-lane logic on machines without a GPU."""
import pytest

from harness import App, OracleError
from kgen_host import KGenHostEngine
from test_oracle_reference_kat import KAT, OUT_OF_SCOPE, check_rows, run_fixture

FIXTURES = [f for f in KAT["fixtures"] if f["id"] not in OUT_OF_SCOPE]


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_kgen_host_matches_oracle(fx):
    try:
        o, orows = run_fixture(fx)
    except OracleError:
        pytest.skip("the reference engine throws on this stream")
    g, grows = run_fixture(fx, engine_factory=lambda blob: KGenHostEngine(blob))
    assert g.matches == o.matches
    check_rows(fx, grows)


def _fuzz_case(seed, partition):
    from fuzz_apps import random_app, random_events
    from siddhi_amd.ql import SiddhiAppCreationException, SiddhiParserException
    src = random_app(seed, partition=partition)
    try:
        o = App(src)
    except (SiddhiAppCreationException, SiddhiParserException):
        return None
    g = App(src, engine_factory=lambda blob: KGenHostEngine(blob))
    for stream, row, t in random_events(seed):
        try:
            o.send(stream, [row], [t])
        except OracleError:
            return None  # the reference would throw: out of the comparable domain
        try:
            g.send(stream, [row], [t])
        except RuntimeError as ex:
            if "capacity" in str(ex):
                return "capacity"
            raise
    return o, g


@pytest.mark.parametrize("seed", range(120))
def test_kgen_host_fuzz(seed):
    r = _fuzz_case(seed, partition=seed % 3 == 0)
    if r is None:
        pytest.skip("app rejected by the planner or the reference would throw")
    if r == "capacity":
        pytest.skip("instance pools exceeded (loud SDH_E_CAPACITY on the device)")
    o, g = r
    assert g.matches == o.matches
