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


def _entries(cache, n):
    clen = int.from_bytes(cache[22:24], "big")
    body = cache[24 + clen:]
    return [(body[i // 4] >> (2 * (i % 4))) & 3 for i in range(n)]


@pytest.mark.parametrize("mode", ["bridge", "client", "server", "first", "router"])
@pytest.mark.parametrize("filt,kept", [("--include=P:5-60", lambda k: 5 <= k <= 60),
                                        ("--exclude=P:1-9,30-31,100-", lambda k: not (k <= 9 or 30 <= k <= 31 or k >= 100))])
def test_auto_with_a_packet_list_adds_the_first_pass_entries(mode, filt, kept):
    """--auto with a packet list: both passes add a DONT_SEND entry for a filtered record
    (tcpprep.c:362-375), the first pass before the second pass's entries (add_cache appends
    to one list, cache.c:246-314; write_cache writes all of it, :146-219): the file holds F
    zero entries, then the N records' entries with the filtered ones zero; the header counts N
    (the second pass's records, tcpprep.c:149,194)"""
    pcap = T.test_pcap()
    args = ["--no-arg-comment", f"--auto={mode}", filt]
    c, ent = oracle_lib.tcpprep(pcap, args, with_entries=True)
    n = int.from_bytes(c[12:20], "big")
    f = sum(1 for k in range(1, n + 1) if not kept(k))
    assert f > 0 and ent == n + f and len(c) == 24 + (n + f + 3) // 4
    e = _entries(c, n + f)
    assert e[:f] == [0] * f
    assert all((e[f + k - 1] == 0) == (not kept(k)) for k in range(1, n + 1))
    # a list that keeps every record is no filter
    full = oracle_lib.tcpprep(pcap, ["--no-arg-comment", f"--auto={mode}", f"--include=P:1-{n}"])
    assert full == oracle_lib.tcpprep(pcap, ["--no-arg-comment", f"--auto={mode}"])
