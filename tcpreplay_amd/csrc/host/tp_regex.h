/* tp_regex.h -- tcpprep --regex compiled to a DFA for the device (tp_regex.c) */
#ifndef TP_REGEX_H
#define TP_REGEX_H
#include <stddef.h>
#include "tp_dev_cfg.h"

/* compile an ERE (REG_EXTENDED | REG_NOSUB, as tcpprep_opts.def:225) into D; on error
   writes the message (the reference's "Unable to compile regex: ..." for a pattern
   regcomp refuses) and returns -1 */
int tp_regex_compile(const char *re, tp_dfa_t *D, char *err, size_t errlen);
/* the DFA's verdict on one string: 1 match, 0 none, -1 a character outside the alphabet */
int tp_dfa_match(const tp_dfa_t *D, const char *s);
/* test entry point (exported): compile `re` and match `s`; -1 when the regex is refused */
int tcpprep_regex_dfa_match(const char *re, const char *s);
#endif
