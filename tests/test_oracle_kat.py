"""The CPU oracle against the hand-traced known-answer cases of SURVEY §8(c)."""
import pytest

import kat_cases


@pytest.mark.parametrize("case", kat_cases.ALL, ids=lambda f: f.__name__)
def test_oracle_kat(case, mk_oracle):
    case(mk_oracle)
