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


SERVICES = "# services\nhttp\t\t80/tcp\t\twww\ndomain 53/udp\nalt 8080/TCP # upper case: matched, then skipped\nbig 70000/udp\n"


def test_oracle_services_file_replaces_the_default_ports(tmp_path):
    f = tmp_path / "services"
    f.write_text(SERVICES)
    pcap = T.test_pcap()
    dflt = oracle_lib.tcpprep(pcap, ["--no-arg-comment", "--port"])
    svc = oracle_lib.tcpprep(pcap, ["--no-arg-comment", "--port", f"--services={f}"])
    assert dflt == T.golden("port") and svc != dflt and len(svc) == len(dflt)
    with pytest.raises(ValueError):
        oracle_lib.tcpprep(pcap, ["--port", f"--services={tmp_path / 'missing'}"])
