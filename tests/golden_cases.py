"""The reference's own tcprewrite golden cases (test/Makefile.am:162-213, the
little-endian `standard_littleendian` target whose outputs are test/test2.*).

Each case: (golden file, input file, cache file or None, argument list, in_scope).
Inputs and expected outputs are the reference's fixtures, copied verbatim under
tests/golden/.  Every case is in scope: the user and hdlc encoders (SURVEY.md §8(f)
rank 3) and --fuzz-seed (rank 4) included.
"""
import os

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CASES = [
    ("test2.rewrite_seed", "test.pcap", None, ["--seed=55"], True),
    ("test2.rewrite_tos", "test.pcap", None, ["--tos=50"], True),
    ("test2.rewrite_portmap", "test.pcap", None, ["--portmap=80:8080"], True),
    ("test2.rewrite_range_portmap", "test.pcap", None, ["--portmap=1-100:49148"], True),
    ("test2.rewrite_sequence", "test.pcap", None, ["--tcp-sequence", "42"], True),
    ("test2.rewrite_endpoint", "test.pcap", "test.auto_router", ["--endpoints=10.10.0.1:10.10.0.2"], True),
    ("test2.rewrite_pnat", "test.pcap", None, ["--pnat=96.17.211.0/24:172.16.0.0/24"], True),
    ("test2.rewrite_pad", "test.pcap", None, ["--fixlen=pad"], True),
    ("test2.rewrite_trunc", "test.pcap", None, ["--fixlen=trunc"], True),
    ("test2.rewrite_mac", "test.pcap", "test.auto_router",
     ["--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
      "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16"], True),
    ("test2.rewrite_enet_subsmac", "test.pcap", None,
     ["--enet-subsmac=00:1f:f3:3c:e1:13,00:22:33:44:55:66",
      "--enet-subsmac=f8:1e:df:e5:84:3a,00:66:55:44:33:22"], True),
    ("test2.rewrite_mac_seed", "test.pcap", None, ["--enet-mac-seed=42"], True),
    ("test2.rewrite_mac_seed_keep", "test.pcap", None,
     ["--enet-mac-seed=42", "--enet-mac-seed-keep-bytes=3"], True),
    ("test2.rewrite_layer2", "test.pcap", None,
     ["--dlt=user", "--user-dlink=00,50,da,5d,46,55,0,7,eb,30,a4,c3,08,0"], True),
    ("test2.rewrite_config", "test.pcap", None,
     ["--enet-vlan=add", "--enet-vlan-tag=45", "--enet-vlan-cfi=1", "--enet-vlan-pri=5"], True),
    ("test2.rewrite_skip", "test.pcap", "test.auto_router",
     ["--skipbroadcast", "--skipl2broadcast", "--skip-soft-errors", "--seed", "55",
      "--enet-dmac=00:12:13:14:15:16,00:22:33:44:55:66",
      "--enet-smac=00:22:33:44:55:66,00:12:13:14:15:16"], True),
    ("test2.rewrite_dltuser", "test.pcap", None,
     ["--dlt=user", "--user-dlink=0x0f,0x00,0x08,0x00", "--user-dlt=104"], True),
    ("test2.rewrite_dlthdlc", "test.pcap", None,
     ["--dlt=hdlc", "--hdlc-control=0", "--hdlc-address=0x0F"], True),
    ("test2.rewrite_vlan802.1ad", "test.pcap", None,
     ["--enet-vlan=add", "--enet-vlan-tag=42", "--enet-vlan-cfi=1", "--enet-vlan-pri=2",
      "--enet-vlan-proto=802.1ad"], True),
    ("test2.rewrite_vlandel", "test.rewrite_config", None, ["--enet-vlan=del"], True),
    ("test2.rewrite_efcs", "test.pcap", None, ["--efcs"], True),
    ("test2.rewrite_1ttl", "test.pcap", None, ["--ttl=58"], True),
    ("test2.rewrite_2ttl", "test.pcap", None, ["--ttl=+58"], True),
    ("test2.rewrite_3ttl", "test.pcap", None, ["--ttl=-58"], True),
    ("test2.rewrite_1ttl-hdrfix", "test.pcap", None, ["--ttl=59", "--fixhdrlen"], True),
    ("test2.rewrite_2ttl-hdrfix", "test.pcap", None, ["--ttl=+59", "--fixhdrlen"], True),
    ("test2.rewrite_3ttl-hdrfix", "test.pcap", None, ["--ttl=-59", "--fixhdrlen"], True),
    ("test2.rewrite_mtutrunc", "test.pcap", None, ["--mtu-trunc", "--mtu=300"], True),
    ("test2.rewrite_l7fuzzing", "test.pcap", None, ["--fuzz-seed=42", "--fuzz-factor=2"], True),
    ("test2.rewrite_fixcsum", "test.pcap", None, ["--fixcsum"], True),
    ("test2.rewrite_fixlen_pad", "test.pcap", None, ["--fixlen=pad"], True),
    ("test2.rewrite_fixlen_trunc", "test.pcap", None, ["--fixlen=trunc"], True),
    ("test2.rewrite_fixlen_del", "test.pcap", None, ["--fixlen=del"], True),
]

IN_SCOPE = [c for c in CASES if c[4]]


def read(name):
    with open(os.path.join(GOLDEN_DIR, name), "rb") as f:
        return f.read()
