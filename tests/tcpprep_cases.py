"""tcpprep golden cases: the argument lines of the reference's test/Makefile.am:87-104
(tcpprep run with --no-arg-comment on test/test.pcap; the regex lines at :96,100), in long-option form, and the
cache files they produced (tests/golden/prep.*, copied from the reference's test/)."""
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = {
    "cidr": ["--cidr=96.17.211.0/24"],
    "cidr_reverse": ["--cidr=96.17.211.0/24", "--reverse"],
    "mac": ["--mac=00:1f:f3:3c:e1:13"],
    "mac_reverse": ["--mac=00:1f:f3:3c:e1:13", "--reverse"],
    "port": ["--port"],
    "comment": ["--comment=This is a comment", "--port"],
    "exclude_packets": ["--cidr=96.17.211.0/24", "--exclude=P:61-65,88-91"],
    "include_packets": ["--cidr=96.17.211.0/24", "--include=P:61-65,88-91"],
    "include_source": ["--cidr=96.17.211.0/24", "--include=S:96.0.0.0/8"],
    "include_dest": ["--cidr=96.17.211.0/24", "--include=D:96.0.0.0/8"],
    "auto_bridge": ["--auto=bridge"],
    "auto_client": ["--auto=client"],
    "auto_server": ["--auto=server"],
    "auto_first": ["--auto=first"],
    "auto_router": ["--auto=router"],
    "regex": ["--regex=96.17.211.*"],
    "regex_reverse": ["--regex=96.17.211.*", "--reverse"],
}


def args(name):
    return ["--no-arg-comment"] + CASES[name]


def golden(name):
    with open(os.path.join(GOLDEN, "prep." + name), "rb") as f:
        return f.read()


def test_pcap():
    with open(os.path.join(GOLDEN, "test.pcap"), "rb") as f:
        return f.read()
