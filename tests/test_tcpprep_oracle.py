"""The tcpprep oracle (oracle/tcpprep_oracle.c) pinned on the reference's own cache
files (test/Makefile.am:93-104 -> tests/golden/prep.*).  CPU only."""
import pytest

import oracle_lib
import tcpprep_cases as T


@pytest.mark.parametrize("name", sorted(T.CASES))
def test_oracle_matches_reference_cache(name):
    assert oracle_lib.tcpprep(T.test_pcap(), T.args(name)) == T.golden(name)


def test_oracle_rejects_unknown_option():
    with pytest.raises(ValueError):
        oracle_lib.tcpprep(T.test_pcap(), ["--auto=bogus"])
