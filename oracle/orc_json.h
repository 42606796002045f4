/* orc_json.h -- oracle JSON DOM (TEST INFRASTRUCTURE, see otm_oracle.h) */
#ifndef ORC_JSON_H
#define ORC_JSON_H
#include <stddef.h>
#include <stdint.h>

typedef struct sbuf {
  char* p;
  size_t len, cap;
} sbuf;
void sb_init(sbuf* b);
void sb_put(sbuf* b, const char* s, size_t n);
void sb_puts(sbuf* b, const char* s);
void sb_printf(sbuf* b, const char* fmt, ...);

enum { JV_NULL = 0, JV_BOOL, JV_INT, JV_FLOAT, JV_STR, JV_ARR, JV_OBJ };
typedef struct jv {
  int t;
  int bigint; /* JV_FLOAT holding an int beyond int64; digits in s */
  int64_t i;  /* INT, BOOL */
  double d;   /* FLOAT */
  char* s;    /* STR (UTF-8) */
  size_t slen;
  struct jv** items; /* ARR / OBJ values */
  char** keys;       /* OBJ */
  size_t* klens;
  size_t n, cap;
} jv;

jv* jv_new(int t);
jv* jv_int(int64_t i);
jv* jv_float(double d);
jv* jv_bool(int b);
jv* jv_str(const char* s, size_t n);
void jv_free(jv* v);
void jv_push(jv* arr, jv* x);
void jv_set(jv* obj, const char* k, size_t kn, jv* x);
jv* jv_get(const jv* obj, const char* k);
void jv_del(jv* obj, const char* k);
const char* jv_typename(const jv* v);

jv* json_parse(const char* s, size_t n, char** err);
char* utf8_check(const unsigned char* s, size_t n);
void json_write(sbuf* b, const jv* v);
void py_float_repr(sbuf* b, double d);

#endif
