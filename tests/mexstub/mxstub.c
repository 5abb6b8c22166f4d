/*
 * mxstub.c -- TEST INFRASTRUCTURE ONLY: the MATLAB matrix / MEX API subset declared in
 * tests/mexstub/mex.h, so tests/test_mex.py can run the MEX drop-ins (mex/BuildAwG.c,
 * mex/Buildxhat.c, mex/BuildRSD.c) against libfba.so without MATLAB.  mexErrMsgIdAndTxt unwinds to
 * mxstub_call (setjmp / longjmp), as MATLAB aborts the MEX call.
 */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

enum { K_DOUBLE, K_INT32, K_CHAR, K_CELL, K_STRUCT };

struct mxArray_tag {
    int kind;
    size_t m, n;
    void* data;        /* double / int32 elements, or the char string (NUL-terminated) */
    mxArray** elems;   /* cell elements, or struct values [element * nf + field] */
    int nf;
    char** fnames;
};

static mxArray* alloc_arr(int kind, size_t m, size_t n) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->kind = kind;
    a->m = m;
    a->n = n;
    return a;
}

size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
size_t mxGetNumberOfElements(const mxArray* a) { return a->kind == K_CHAR ? (a->data ? strlen((char*)a->data) : 0) : a->m * a->n; }
int mxIsDouble(const mxArray* a) { return a && a->kind == K_DOUBLE; }
int mxIsInt32(const mxArray* a) { return a && a->kind == K_INT32; }
int mxIsChar(const mxArray* a) { return a && a->kind == K_CHAR; }
int mxIsCell(const mxArray* a) { return a && a->kind == K_CELL; }
int mxIsStruct(const mxArray* a) { return a && a->kind == K_STRUCT; }
int mxIsClass(const mxArray* a, const char* c) {
    static const char* names[] = {"double", "int32", "char", "cell", "struct"};
    return a && strcmp(names[a->kind], c) == 0;
}
double* mxGetDoubles(const mxArray* a) { return a->kind == K_DOUBLE ? (double*)a->data : NULL; }
mxInt32* mxGetInt32s(const mxArray* a) { return a->kind == K_INT32 ? (mxInt32*)a->data : NULL; }
double mxGetScalar(const mxArray* a) {
    if (a->kind == K_DOUBLE && a->m * a->n > 0) return ((double*)a->data)[0];
    if (a->kind == K_INT32 && a->m * a->n > 0) return ((int32_t*)a->data)[0];
    return 0.0;
}
mxArray* mxGetField(const mxArray* a, mwIndex i, const char* name) {
    if (!a || a->kind != K_STRUCT || i >= a->m * a->n) return NULL;
    for (int f = 0; f < a->nf; ++f)
        if (strcmp(a->fnames[f], name) == 0) return a->elems[i * a->nf + f];
    return NULL;
}
mxArray* mxGetCell(const mxArray* a, mwIndex i) { return (a->kind == K_CELL && i < a->m * a->n) ? a->elems[i] : NULL; }
char* mxArrayToString(const mxArray* a) {
    if (a->kind != K_CHAR) return NULL;
    const char* s = a->data ? (const char*)a->data : "";
    char* r = (char*)malloc(strlen(s) + 1);
    strcpy(r, s);
    return r;
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
    (void)c;
    mxArray* a = alloc_arr(K_DOUBLE, m, n);
    a->data = calloc(m * n + 1, sizeof(double));
    return a;
}
mxArray* mxCreateDoubleScalar(double v) {
    mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
    ((double*)a->data)[0] = v;
    return a;
}
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID c, mxComplexity x) {
    (void)x;
    size_t n = 1;
    for (mwSize d = 1; d < nd; ++d) n *= dims[d];
    mxArray* a = alloc_arr(c == mxINT32_CLASS ? K_INT32 : K_DOUBLE, nd ? dims[0] : 0, n);
    a->data = calloc(a->m * a->n + 1, c == mxINT32_CLASS ? sizeof(int32_t) : sizeof(double));
    return a;
}
mxArray* mxCreateCellMatrix(mwSize m, mwSize n) {
    mxArray* a = alloc_arr(K_CELL, m, n);
    a->elems = (mxArray**)calloc(m * n + 1, sizeof(mxArray*));
    return a;
}
mxArray* mxCreateString(const char* s) {
    mxArray* a = alloc_arr(K_CHAR, 1, strlen(s));
    a->data = malloc(strlen(s) + 1);
    strcpy((char*)a->data, s);
    return a;
}
mxArray* mxCreateStructMatrix(mwSize m, mwSize n, int nf, const char** names) {
    mxArray* a = alloc_arr(K_STRUCT, m, n);
    a->nf = nf;
    a->fnames = (char**)calloc(nf + 1, sizeof(char*));
    for (int f = 0; f < nf; ++f) {
        a->fnames[f] = (char*)malloc(strlen(names[f]) + 1);
        strcpy(a->fnames[f], names[f]);
    }
    a->elems = (mxArray**)calloc(m * n * nf + 1, sizeof(mxArray*));
    return a;
}
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    if (a->kind == K_CELL)
        for (size_t i = 0; i < a->m * a->n; ++i) mxDestroyArray(a->elems[i]);
    if (a->kind == K_STRUCT) {
        for (size_t i = 0; i < a->m * a->n * a->nf; ++i) mxDestroyArray(a->elems[i]);
        for (int f = 0; f < a->nf; ++f) free(a->fnames[f]);
        free(a->fnames);
    }
    free(a->elems);
    free(a->data);
    free(a);
}
void mxSetCell(mxArray* a, mwIndex i, mxArray* v) {
    mxDestroyArray(a->elems[i]);
    a->elems[i] = v;
}
void mxSetField(mxArray* a, mwIndex i, const char* name, mxArray* v) {
    for (int f = 0; f < a->nf; ++f)
        if (strcmp(a->fnames[f], name) == 0) {
            mxDestroyArray(a->elems[i * a->nf + f]);
            a->elems[i * a->nf + f] = v;
            return;
        }
}
mxArray* mxDuplicateArray(const mxArray* a) {
    if (!a) return NULL;
    mxArray* b = alloc_arr(a->kind, a->m, a->n);
    if (a->kind == K_DOUBLE || a->kind == K_INT32) {
        const size_t es = a->kind == K_DOUBLE ? sizeof(double) : sizeof(int32_t);
        b->data = calloc(a->m * a->n + 1, es);
        memcpy(b->data, a->data, a->m * a->n * es);
    } else if (a->kind == K_CHAR) {
        b->data = malloc(strlen((char*)a->data) + 1);
        strcpy((char*)b->data, (char*)a->data);
    } else if (a->kind == K_CELL) {
        b->elems = (mxArray**)calloc(a->m * a->n + 1, sizeof(mxArray*));
        for (size_t i = 0; i < a->m * a->n; ++i) b->elems[i] = mxDuplicateArray(a->elems[i]);
    } else {
        b->nf = a->nf;
        b->fnames = (char**)calloc(a->nf + 1, sizeof(char*));
        for (int f = 0; f < a->nf; ++f) {
            b->fnames[f] = (char*)malloc(strlen(a->fnames[f]) + 1);
            strcpy(b->fnames[f], a->fnames[f]);
        }
        b->elems = (mxArray**)calloc(a->m * a->n * a->nf + 1, sizeof(mxArray*));
        for (size_t i = 0; i < a->m * a->n * a->nf; ++i) b->elems[i] = mxDuplicateArray(a->elems[i]);
    }
    return b;
}
void* mxMalloc(size_t n) { return malloc(n ? n : 1); }
void* mxCalloc(size_t n, size_t s) { return calloc(n ? n : 1, s ? s : 1); }
void mxFree(void* p) { free(p); }

static jmp_buf g_jmp;
static int g_armed = 0;
static char g_err[1024];
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    int k = snprintf(g_err, sizeof g_err, "%s: ", id);
    vsnprintf(g_err + k, sizeof g_err - (size_t)k, fmt, ap);
    va_end(ap);
    if (g_armed) longjmp(g_jmp, 1);
    fprintf(stderr, "%s\n", g_err);
    abort();
}
int mexPrintf(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int r = vprintf(fmt, ap);
    va_end(ap);
    fflush(stdout);
    return r;
}
static void (*g_atexit[16])(void);  /* one per loaded MEX library (MATLAB keeps one per MEX file) */
static int g_natexit = 0;
int mexAtExit(void (*f)(void)) {
    for (int i = 0; i < g_natexit; ++i)
        if (g_atexit[i] == f) return 0;
    if (g_natexit < 16) g_atexit[g_natexit++] = f;
    return 0;
}
/* the two conversions the drop-ins ask MATLAB for: cellstr() and char() of already-converted inputs */
int mexCallMATLAB(int nl, mxArray* pl[], int nr, mxArray* pr[], const char* name) {
    if (nl < 1 || nr < 1) return 1;
    if (strcmp(name, "cellstr") == 0 && pr[0]->kind == K_CELL) { pl[0] = mxDuplicateArray(pr[0]); return 0; }
    if (strcmp(name, "char") == 0 && pr[0]->kind == K_CHAR) { pl[0] = mxDuplicateArray(pr[0]); return 0; }
    return 1;
}

/* ---- harness entry points (ctypes) ---- */
typedef void (*mexfn)(int, mxArray*[], int, const mxArray*[]);
int mxstub_call(mexfn f, int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs) {
    g_armed = 1;
    g_err[0] = 0;
    if (setjmp(g_jmp)) {
        g_armed = 0;
        return 1;
    }
    f(nlhs, plhs, nrhs, prhs);
    g_armed = 0;
    return 0;
}
const char* mxstub_error(void) { return g_err; }
void mxstub_exit(void) {
    for (int i = 0; i < g_natexit; ++i) g_atexit[i]();
    g_natexit = 0;
}
