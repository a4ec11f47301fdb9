#!/bin/sh
# Regenerates tests/golden/autoopts_layout.json: the field offsets of libopts' option
# descriptors, compiled from the reference's own header (libopts/autoopts/options.h,
# configured with the HAVE_* switches the header itself offers for test compilations).
# Run in the build container, where /root/reference exists; the JSON is the fixture.
set -e
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
T=$(mktemp -d)
cat > "$T/probe.c" <<'PROBE'
#include <stddef.h>
#include <stdio.h>
#include "autoopts/options.h"
int main(void)
{
    printf("{\"sizeof_opt_desc\": %zu, \"optOccCt\": %zu, \"fOptState\": %zu, \"optArg\": %zu, "
           "\"optCookie\": %zu, \"pz_NAME\": %zu, \"pz_Name\": %zu, \"pOptDesc\": %zu, \"specOptIdx\": %zu, "
           "\"optCt\": %zu, \"apzArgs\": %zu, \"OPTST_SET_MASK\": %u, \"OPTST_ARG_TYPE_MASK\": %u, "
           "\"OPARG_TYPE_NUMERIC\": %d, \"OPARG_TYPE_STRING\": %d}\n",
           sizeof(tOptDesc), offsetof(tOptDesc, optOccCt), offsetof(tOptDesc, fOptState), offsetof(tOptDesc, optArg),
           offsetof(tOptDesc, optCookie), offsetof(tOptDesc, pz_NAME), offsetof(tOptDesc, pz_Name),
           offsetof(tOptions, pOptDesc), offsetof(tOptions, specOptIdx), offsetof(tOptions, optCt),
           offsetof(tArgList, apzArgs), OPTST_SET_MASK, OPTST_ARG_TYPE_MASK, OPARG_TYPE_NUMERIC, OPARG_TYPE_STRING);
    return 0;
}
PROBE
gcc -DHAVE_STDINT_H -DHAVE_STDBOOL_H -DHAVE_LIMITS_H -DHAVE_SYSEXITS_H -I"$REF/libopts" -o "$T/probe" "$T/probe.c"
"$T/probe" > "$HERE/autoopts_layout.json"
rm -rf "$T"
cat "$HERE/autoopts_layout.json"
