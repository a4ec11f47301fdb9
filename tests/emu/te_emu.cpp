// te_emu.cpp -- TEST INFRASTRUCTURE ONLY.  The generic lane's per-record edit
// (tcpreplay_amd/csrc/kernels/edit_pkt.hpp tcpedit_packet, the code te_edit_tiles runs
// one lane per record) compiled for the host, so the CPU suite can drive it record by
// record under AddressSanitizer and compare it with the oracle before a GPU sees it.
// It is never part of the product: libtcpedit_hip.so edits on the GPU only, and nothing
// under tcpreplay_amd/ loads this program.
//
// Each record gets a slot laid out as tile_body (tcpedit_kernels.hip) lays it out:
// [headroom cfg.slot_head][alignment gap g][16-byte record header][data][16 zeroed bytes],
// rounded to 16 -- in its own heap block, so a move of the record header past the
// headroom, or a write past the slot, is an ASan report rather than silent corruption.
// The headroom and gap hold garbage (the LDS there holds other records' bytes).
//
// usage: te_emu CFG PORTLUT|- IN.pcap DIRBITS|- SLOT(0|1) OUT.pcap
//   CFG: the te_dev_cfg_t bytes (tcpedit_get_dev_cfg); PORTLUT: 65536 u16 or "-";
//   DIRBITS: the tcpprep cache body or "-".  Native-order microsecond pcap input.
//   Prints "records R written W unsupported U error E fuzz_state S".
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "edit_pkt.hpp"

using namespace te;

static std::vector<uint8_t> slurp(const char *path) {
    std::vector<uint8_t> v;
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror(path);
        exit(2);
    }
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
    fclose(f);
    return v;
}

template <bool FZ, bool AD>
static int edit(Pkt &pk, const te_dev_cfg_t &cfg, const uint16_t *lut, int dir, bool &warned, uint32_t mode,
                uint32_t st) {
    return tcpedit_packet<FZ, AD>(pk, cfg, lut, dir, warned, mode, st);
}

int main(int argc, char **argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: te_emu CFG PORTLUT|- IN.pcap DIRBITS|- SLOT OUT.pcap\n");
        return 2;
    }
    const std::vector<uint8_t> cfgb = slurp(argv[1]);
    if (cfgb.size() != sizeof(te_dev_cfg_t)) {
        fprintf(stderr, "config: %zu bytes, te_dev_cfg_t is %zu\n", cfgb.size(), sizeof(te_dev_cfg_t));
        return 2;
    }
    te_dev_cfg_t cfg;
    memcpy(&cfg, cfgb.data(), sizeof cfg);
    std::vector<uint16_t> lut(65536);
    for (int p = 0; p < 65536; ++p) lut[p] = (uint16_t)p;
    if (strcmp(argv[2], "-")) {
        const std::vector<uint8_t> l = slurp(argv[2]);
        if (l.size() != 131072) return 2;
        memcpy(lut.data(), l.data(), l.size());
    }
    const std::vector<uint8_t> img = slurp(argv[3]);
    std::vector<uint8_t> dirbits;
    const bool have_dir = strcmp(argv[4], "-") != 0;
    if (have_dir) dirbits = slurp(argv[4]);
    const bool slot_mode = atoi(argv[5]) != 0;
    const bool fz = cfg.fuzz_seed != 0;
    const bool ad = cfg.decoder != TE_DEC_EN10MB || cfg.encoder == TE_ENC_NOENC || cfg.encoder == TE_ENC_PPP;
    const uint32_t head = slot_mode ? cfg.slot_head : 0u;
    if (img.size() < 24) return 2;
    std::vector<uint8_t> out(img.begin(), img.begin() + 24);
    uint32_t fstate = cfg.fuzz_seed;  // fuzzing_init (fuzzing.c:12-20)
    // DLT_JUNIPER_ETHER: the decoder state the last whole inner decode left (what a frame
    // whose extensions are not Ethernet is encoded with), as te_jnpr_mark + its scan give it
    te_jstate_t jst{};
    bool jvalid = false;
    uint64_t recs = 0, written = 0, unsup = 0;
    int error = 0;
    size_t off = 24;
    while (off + 16 <= img.size()) {
        const uint8_t *rec = img.data() + off;
        const uint32_t caplen = ld32(rec + 8), len = ld32(rec + 12);
        if (caplen > MAX_SNAPLEN || off + 16 + caplen > img.size()) break;  // libpcap's stop
        if (len > MAX_SNAPLEN) {  // tcprewrite.c:296-297
            error = 1;
            break;
        }
        uint32_t data = caplen;
        if (cfg.fixlen == TE_FIXLEN_PAD && len > data) data = len;
        const uint32_t g = slot_mode ? (uint32_t)(off & 15) : 0u;
        const uint32_t slot = slot_mode ? TE_SLOT_BYTES_OF_H(head, g, data) : 16u + caplen;
        const uint64_t pktno = recs;
        int dir = TE_DIR_C2S;
        if (have_dir) {  // check_cache (cache.c:321-354)
            const uint64_t idx = pktno >> 2;
            const uint32_t bit = (uint32_t)((pktno & 3) * 2) + 1;
            const uint8_t b = idx < dirbits.size() ? dirbits[idx] : 0;
            dir = !(b & (1u << bit)) ? TE_DIR_NOSEND : ((b & (1u << (bit - 1))) ? TE_DIR_C2S : TE_DIR_S2C);
        }
        // this record's first decode, on its input bytes (te_jnpr_mark): whole or not
        bool jwhole = false;
        te_jstate_t jnext{};
        if (cfg.decoder == TE_DEC_JNPR && dir != TE_DIR_NOSEND) {
            std::vector<uint8_t> tmp(rec + 16, rec + 16 + caplen);
            tmp.resize(caplen + 64);
            Pkt q;
            q.d = tmp.data();
            q.caplen = caplen;
            if (cfg.efcs && len > 4 && caplen == len) q.caplen -= 4;
            q.len = len;
            q.phys = q.avail = q.ext = q.caplen;
            q.unsupported = false;
            q.need = 0;
            q.strict = false;
            uint32_t hl = 0;
            Dec ds;
            ds.dst_modified = false;
            jwhole = decoder_proto(q, cfg) >= 0 && jnpr_header(q.d, q.caplen, hl) == RC_OK &&
                     foreign_decode(q, cfg, ds) == RC_OK;
            if (jwhole) {
                for (int i = 0; i < 6; ++i) {
                    jnext.dstaddr[i] = ds.dstaddr[i];
                    jnext.srcaddr[i] = ds.srcaddr[i];
                }
                jnext.proto = (uint16_t)ds.proto;
                jnext.vlan_tag = ds.vlan_tag;
                jnext.vlan_pri = ds.vlan_pri;
                jnext.vlan_cfi = ds.vlan_cfi;
                jnext.vlan_proto = ds.vlan_proto;
                jnext.vlan_offset = ds.vlan_offset;
                jnext.vlan = (uint8_t)ds.vlan;
            }
        }
        bool reached = false;
        int rc = RC_OK;
        bool warned = false;
        Pkt pk;
        uint8_t *buf = nullptr;
        for (int pass = fz ? 0 : 1; pass < 2; ++pass) {
            free(buf);
            buf = (uint8_t *)malloc(slot);
            memset(buf, 0xA5, slot);  // garbage before the record (another record's LDS bytes)
            const uint32_t r0 = head + g;
            memcpy(buf + r0, rec, 16 + caplen);
            memset(buf + r0 + 16 + caplen, 0, slot - (r0 + 16 + caplen));
            pk = Pkt();
            pk.d = buf + r0 + 16;
            pk.caplen = caplen;
            pk.len = len;
            pk.phys = caplen;
            pk.avail = slot - (r0 + 16);
            pk.unsupported = false;
            pk.need = 0;
            pk.ext = caplen;
            pk.strict = false;
            pk.room = r0;
            pk.l2carry = 0;
            pk.defer = false;
            pk.jc = jvalid ? &jst : nullptr;
            pk.jnone = !jvalid;
            // (a fuzzed record's second decode: the state after its own first pass)
            pk.jc2 = jwhole ? &jnext : pk.jc;
            pk.jnone2 = !jwhole && !jvalid;
            if (dir == TE_DIR_NOSEND) break;  // tcprewrite.c:314-315: written unedited
            const uint32_t mode = !fz ? TE_FUZZ_OFF : pass == 0 ? TE_FUZZ_PROBE : TE_FUZZ_APPLY;
            const uint32_t st = pass == 1 && reached ? fstate : 0u;
            if (fz && ad) rc = edit<true, true>(pk, cfg, lut.data(), dir, warned, mode, st);
            else if (fz) rc = edit<true, false>(pk, cfg, lut.data(), dir, warned, mode, st);
            else if (ad) rc = edit<false, true>(pk, cfg, lut.data(), dir, warned, mode, st);
            else rc = edit<false, false>(pk, cfg, lut.data(), dir, warned, mode, st);
            if (pass == 0) reached = rc == RC_REACHED;
        }
        if (reached) tcpr_random_dev(fstate);  // the record's draw (fuzzing.c:88)
        if (jwhole) {
            jst = jnext;
            jvalid = true;
        }
        ++recs;
        bool write = true;
        if (rc == RC_ERROR) {
            error = 1;
            free(buf);
            break;  // the host truncates the output at the first hard error
        }
        if (rc == RC_SOFT && cfg.skip_soft_errors) write = false;
        if (write && pk.caplen == 0) write = false;
        if (pk.unsupported && write) ++unsup;
        if (write) {
            uint8_t *orec = pk.d - 16;
            st32(orec, ld32(rec));
            st32(orec + 4, ld32(rec + 4));
            st32(orec + 8, pk.caplen);
            st32(orec + 12, pk.len);
            out.insert(out.end(), orec, orec + 16 + pk.caplen);
            ++written;
        }
        free(buf);
        off += 16 + caplen;
    }
    st32(out.data() + 20, (uint32_t)cfg.out_linktype);
    FILE *f = fopen(argv[6], "wb");
    if (!f || fwrite(out.data(), 1, out.size(), f) != out.size()) return 2;
    fclose(f);
    printf("records %llu written %llu unsupported %llu error %d fuzz_state %u\n", (unsigned long long)recs,
           (unsigned long long)written, (unsigned long long)unsup, error, fstate);
    return 0;
}
