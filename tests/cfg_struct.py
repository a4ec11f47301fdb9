"""ctypes mirror of te_dev_cfg_t (tcpreplay_amd/csrc/include/te_dev_cfg.h) for host tests."""
import ctypes

MAXC, MAXS, MAXPM = 16, 32, 64


class Cidr(ctypes.Structure):
    _fields_ = [("family", ctypes.c_int32), ("masklen", ctypes.c_int32), ("network", ctypes.c_uint32),
                ("network6", ctypes.c_uint8 * 16)]


class CidrMap(ctypes.Structure):
    _fields_ = [("frm", Cidr), ("to", Cidr)]


class DevCfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint8) for n in ("skip_broadcast", "rewrite_ip", "fixcsum", "efcs", "mtu_truncate",
                                               "fixhdrlen", "l2_skip_broadcast", "skip_soft_errors")] + [
        ("fixlen", ctypes.c_int32), ("ttl_mode", ctypes.c_int32), ("ttl_value", ctypes.c_uint32),
        ("tos", ctypes.c_int32), ("flowlabel", ctypes.c_int32), ("tclass", ctypes.c_int32), ("mtu", ctypes.c_int32),
        ("tcp_sequence_enable", ctypes.c_uint32), ("tcp_sequence_adjust", ctypes.c_uint32),
        ("seed", ctypes.c_uint32), ("has_portmap", ctypes.c_int32),
        ("n_cidrmap1", ctypes.c_int32), ("n_cidrmap2", ctypes.c_int32), ("n_srcipmap", ctypes.c_int32),
        ("n_dstipmap", ctypes.c_int32),
        ("cidrmap1", CidrMap * MAXC), ("cidrmap2", CidrMap * MAXC), ("srcipmap", CidrMap * MAXC),
        ("dstipmap", CidrMap * MAXC),
        ("intf1_dmac", ctypes.c_uint8 * 6), ("intf1_smac", ctypes.c_uint8 * 6), ("intf2_dmac", ctypes.c_uint8 * 6),
        ("intf2_smac", ctypes.c_uint8 * 6), ("n_subs", ctypes.c_int32), ("subs", (ctypes.c_uint8 * 12) * MAXS),
        ("random_set", ctypes.c_uint32), ("random_keep", ctypes.c_int32), ("random_mask", ctypes.c_uint8 * 8),
        ("mac_mask", ctypes.c_int32), ("vlan", ctypes.c_int32), ("vlan_tag", ctypes.c_uint32),
        ("vlan_pri", ctypes.c_uint32), ("vlan_cfi", ctypes.c_uint32), ("vlan_proto", ctypes.c_uint32),
        ("n_pm", ctypes.c_int32), ("pm_from", ctypes.c_uint16 * MAXPM), ("pm_to", ctypes.c_uint16 * MAXPM),
        ("encoder", ctypes.c_int32), ("out_linktype", ctypes.c_int32), ("user_length", ctypes.c_int32),
        ("hdlc_address", ctypes.c_uint32), ("hdlc_control", ctypes.c_uint32),
        ("user_l2client", ctypes.c_uint8 * 256), ("user_l2server", ctypes.c_uint8 * 256),
        ("fuzz_seed", ctypes.c_uint32), ("fuzz_factor", ctypes.c_uint32),
        ("decoder", ctypes.c_int32), ("l2carry", ctypes.c_uint32), ("cidr_spill", ctypes.c_uint64 * 4),
        ("slot_head", ctypes.c_uint32), ("pad_", ctypes.c_uint32)]
