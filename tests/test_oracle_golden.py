"""Pin the oracle: it must reproduce every transcribed reference known-answer test.

The fixtures under tests/golden/ are data transcribed from the reference's TestNG
suites (tests/golden/extract_golden.py).  Constructs outside the state path
(group by, select *, inner '#' streams, non-partitioned streams inside a
partition) are listed in OUT_OF_SCOPE.
"""
import pytest

from golden_runner import load_fixtures, run_fixture
from oracle.oracle import OracleEngine

OUT_OF_SCOPE = {
    "AbsentPatternTestCase.testQueryAbsent41": "select * (selector, not the state path)",
    "CountPatternTestCase.testQuery14": "group by (selector)",
    "PatternPartitionTestCase.testPatternPartitionQuery30": "unkeyed stream broadcast into a partition",
    "PatternPartitionTestCase.testPatternPartitionQuery32": "inner '#' streams",
    "PatternPartitionTestCase.testPatternPartitionQuery33": "inner '#' streams",
}

FIXTURES = load_fixtures()


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_oracle_reproduces_reference(fx):
    if fx["name"] in OUT_OF_SCOPE:
        pytest.skip(OUT_OF_SCOPE[fx["name"]])
    ok, msg, _ = run_fixture(fx, OracleEngine)
    assert ok, f'{fx["source"]}: {msg}'


def test_corpus_size():
    assert len(FIXTURES) >= 400
