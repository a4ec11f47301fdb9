// Debugging aid: runs edit_pkt.hpp's per-packet logic on the CPU over a
// contiguous copy of each record (the kernel's CONTIG layout) and prints the
// edited records, for diffing against the oracle.  Not a product path.
#define TE_HOST_EMU 1
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "edit_pkt.hpp"
int main(int argc, char **argv) {
    // usage: host_emu cfg.bin in.pcap [portlut.bin]
    FILE *f = fopen(argv[1], "rb");
    te_dev_cfg_t cfg;
    if (fread(&cfg, sizeof cfg, 1, f) != 1) return 2;
    fclose(f);
    f = fopen(argv[2], "rb");
    std::vector<uint8_t> in(1 << 26);
    size_t n = fread(in.data(), 1, in.size(), f);
    fclose(f);
    std::vector<uint16_t> lut(65536);
    for (int i = 0; i < 65536; i++) lut[i] = i;
    if (argc > 3) { f = fopen(argv[3], "rb"); fread(lut.data(), 2, 65536, f); fclose(f); }
    std::vector<uint8_t> span(in.begin(), in.begin() + n);  // contiguous like the LDS image
    fwrite(in.data(), 1, 24, stdout);
    size_t off = 24;
    while (off + 16 <= n) {
        uint32_t cap, len;
        memcpy(&cap, &span[off + 8], 4);
        memcpy(&len, &span[off + 12], 4);
        te::Pkt pk{&span[off + 16], cap, len, cap, cap, false};
        bool warned;
        int rc = te::tcpedit_packet(pk, cfg, lut.data(), TE_DIR_C2S, warned);
        uint8_t *orec = pk.d - 16;
        memcpy(orec + 8, &pk.caplen, 4);
        memcpy(orec + 12, &pk.len, 4);
        if (rc != te::RC_ERROR && !(rc == te::RC_SOFT && cfg.skip_soft_errors) && pk.caplen) fwrite(orec, 1, 16 + pk.caplen, stdout);
        if (pk.unsupported) fprintf(stderr, "unsupported at %zu\n", off);
        off += 16 + cap;
    }
    return 0;
}
