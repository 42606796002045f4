/* orc_internal.h -- oracle internals (TEST INFRASTRUCTURE, see otm_oracle.h) */
#ifndef ORC_INTERNAL_H
#define ORC_INTERNAL_H
#include "orc_json.h"
#include "otm_oracle.h"

/* Match the trace of a parsed request (uuid + trace[]) and write the
 * {"segments":[...]} JSON.  Returns 0 with *err (malloc'd) on failure. */
int orc_match_dom(const orc_graph* g, const orc_params* p, const jv* req, sbuf* out, char** err);
int dom_report(const orc_report_cfg* rc, const jv* trace, jv* segments, sbuf* out, sbuf* errs, char** exc);

#endif
