/*
 * te_autoopts.c -- the AutoOpts option bridge.
 *
 * The reference's tcpedit_post_args (src/tcpedit/parse_args.c:34-254) reads the
 * tcpedit options through the HAVE_OPT / OPT_ARG / OPT_VALUE_* / STACKCT_OPT /
 * STACKLST_OPT macros of the calling tool's AutoGen-generated option header: every
 * tool that links libtcpedit (tcprewrite, tcpreplay-edit, tcpbridge) includes
 * tcpedit/tcpedit_opts.def into its own option set (tcprewrite_opts.def:50,
 * tcpreplay_opts.def:71, tcpbridge_opts.def:63) and hands its tOptions to
 * optionProcess() (tcprewrite.c:72, tcpreplay.c:66, tcpbridge.c:62).
 *
 * A reference tool relinked against libtcpedit_hip calls tcpedit_post_args with
 * no other option source.  This file finds the tool's option set through weak
 * references to its tOptions object and copies every tcpedit/DLT option that is
 * set into the library's option store, by long name, so the derivation is the
 * same one tcpedit_parse_args feeds.  The two structures are read with the field
 * layout libopts defines (libopts/autoopts/options.h:519-579 struct opt_desc,
 * :603-680 struct options, :194-201 tArgList), restated below.
 *
 * The references are weak and undefined in the library: when the tool's executable
 * defines the object, the link editor exports it to the dynamic symbol table (a
 * shared library on the link line references it) and the loader binds it here;
 * otherwise the address is NULL.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "te_internal.h"

/* options.h:482-491 opt_arg_union_t */
typedef union {
    const char *argString;
    uintptr_t argEnum;
    uintptr_t argIntptr;
    long argInt;
    unsigned long argUint;
    unsigned int argBool;
    void *argFp;
    int argFd;
} te_ao_arg_t;

/* options.h:519-579 struct opt_desc */
typedef struct {
    uint16_t optIndex, optValue, optActualIndex, optActualValue;
    uint16_t optEquivIndex, optMinCt, optMaxCt, optOccCt;
    uint32_t fOptState; /* opt_state_mask_t */
    uint32_t optUsage;
    te_ao_arg_t optArg;
    void *optCookie;
    const int *pOptMust;
    const int *pOptCant;
    void (*pOptProc)(void *, void *);
    const char *pzText;
    const char *pz_NAME;
    const char *pz_Name;
    const char *pz_DisableName;
    const char *pz_DisablePfx;
} te_ao_desc_t;

/* options.h:194-201 tArgList (the stacked arguments behind optCookie) */
typedef struct {
    int useCt;
    int allocCt;
    const char *apzArgs[6]; /* MIN_ARG_ALLOC_CT; grows past the struct */
} te_ao_arglist_t;

/* options.h:603-680 struct options, up to optCt */
typedef struct {
    int structVersion;
    unsigned int origArgCt;
    char **origArgVect;
    uint32_t fOptSet; /* proc_state_mask_t */
    unsigned int curOptIdx;
    char *pzCurOpt;
    const char *pzProgPath, *pzProgName, *pzPROGNAME, *pzRcName, *pzCopyright, *pzCopyNotice, *pzFullVersion;
    const char *const *papzHomeList;
    const char *pzUsageTitle, *pzExplain, *pzDetail;
    te_ao_desc_t *pOptDesc;
    const char *pzBugAddr;
    void *pExtensions;
    void *pSavedState;
    void *pUsageProc;
    void *pTransProc;
    struct {
        uint16_t more_help, save_opts, number_option, default_opt;
    } specOptIdx; /* option_spec_idx_t, options.h:584-590 */
    int optCt;
    int presetOptCt;
} te_ao_options_t;

#define TE_OPTST_SET_MASK 0x000000FU    /* options.h:270: HAVE_OPT = !UNUSED_OPT */
#define TE_OPTST_ARG_TYPE_MASK 0x000F000U /* options.h:287 */
#define TE_OPTST_ARG_TYPE_SHIFT 12
#define TE_OPARG_TYPE_NUMERIC 5         /* options.h:136 */
#define TE_OPARG_TYPE_NONE 0

/* the tools' option sets (the tOptions objects AutoGen emits as <prog>Options) */
extern te_ao_options_t tcprewriteOptions __attribute__((weak));
extern te_ao_options_t tcpreplayOptions __attribute__((weak));
extern te_ao_options_t tcpbridgeOptions __attribute__((weak));

/* for tests: the offsets this file reads, to check against libopts' own layout */
void te_autoopts_layout(size_t *v, int n)
{
    const size_t o[] = {
        sizeof(te_ao_desc_t),
        offsetof(te_ao_desc_t, optOccCt),
        offsetof(te_ao_desc_t, fOptState),
        offsetof(te_ao_desc_t, optArg),
        offsetof(te_ao_desc_t, optCookie),
        offsetof(te_ao_desc_t, pz_NAME),
        offsetof(te_ao_desc_t, pz_Name),
        offsetof(te_ao_options_t, pOptDesc),
        offsetof(te_ao_options_t, specOptIdx),
        offsetof(te_ao_options_t, optCt),
        offsetof(te_ao_arglist_t, apzArgs),
    };
    for (int i = 0; i < n && i < (int)(sizeof(o) / sizeof(o[0])); i++)
        v[i] = o[i];
}

/* the option set of the running tool, or NULL */
static const te_ao_options_t *tool_options(const char **which)
{
    if (&tcprewriteOptions) {
        *which = "tcprewriteOptions";
        return &tcprewriteOptions;
    }
    if (&tcpreplayOptions) {
        *which = "tcpreplayOptions";
        return &tcpreplayOptions;
    }
    if (&tcpbridgeOptions) {
        *which = "tcpbridgeOptions";
        return &tcpbridgeOptions;
    }
    return NULL;
}

static int import_one(tcpedit_t *t, int k, const te_ao_desc_t *d, const char *which)
{
    const unsigned type = (d->fOptState & TE_OPTST_ARG_TYPE_MASK) >> TE_OPTST_ARG_TYPE_SHIFT;
    char num[32];
    if (te_optdefs[k].stacked) {
        /* STACKCT_OPT / STACKLST_OPT: the tArgList behind optCookie */
        const te_ao_arglist_t *al = (const te_ao_arglist_t *)d->optCookie;
        if (!al || al->useCt <= 0) {
            /* a stacked option set once keeps its argument in optArg as well */
            return d->optArg.argString ? tcpedit_set_option(t, te_optdefs[k].name, d->optArg.argString) : 0;
        }
        for (int i = 0; i < al->useCt; i++)
            if (tcpedit_set_option(t, te_optdefs[k].name, al->apzArgs[i]) < 0)
                return -1;
        return 0;
    }
    if (!te_optdefs[k].has_arg)
        return tcpedit_set_option(t, te_optdefs[k].name, NULL);
    if (type == TE_OPARG_TYPE_NUMERIC) { /* OPT_VALUE_<NAME>: the parsed long */
        snprintf(num, sizeof(num), "%ld", d->optArg.argInt);
        return tcpedit_set_option(t, te_optdefs[k].name, num);
    }
    if (!d->optArg.argString) {
        te_seterr(t, "%s: option --%s is set without an argument", which, te_optdefs[k].name);
        return -1;
    }
    return tcpedit_set_option(t, te_optdefs[k].name, d->optArg.argString);
}

int te_autoopts_import(tcpedit_t *t)
{
    const char *which = NULL;
    const te_ao_options_t *o = tool_options(&which);
    if (!o)
        return 0;
    if (!o->pOptDesc || o->optCt <= 0 || o->optCt > 4096) {
        te_seterr(t, "%s: option descriptor table not initialised", which);
        return -1;
    }
    for (int i = 0; i < o->optCt; i++) {
        const te_ao_desc_t *d = &o->pOptDesc[i];
        if (!d->pz_Name || (d->fOptState & TE_OPTST_SET_MASK) == 0)
            continue;
        for (int k = 0; k < OPT__N; k++) {
            if (strcmp(te_optdefs[k].name, d->pz_Name) != 0)
                continue;
            if (import_one(t, k, d, which) < 0)
                return -1;
            break;
        }
    }
    t->opt_src |= TE_SRC_STORE;
    return 1;
}
