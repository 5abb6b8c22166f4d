/*
 * mex.h -- TEST INFRASTRUCTURE ONLY: a stand-in for MATLAB's MEX / matrix API (R2018a interleaved
 * form), enough to compile and RUN the MEX drop-ins under mex/ without MATLAB (tests/test_mex.py).
 * Implemented by tests/mexstub/mxstub.c: doubles, int32, char, cell and struct arrays, column-major.
 */
#ifndef MXSTUB_MEX_H_
#define MXSTUB_MEX_H_
#include <stddef.h>
#include <stdint.h>

typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef size_t mwIndex;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef enum { mxUNKNOWN_CLASS = 0, mxCELL_CLASS, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxVOID_CLASS,
               mxDOUBLE_CLASS, mxSINGLE_CLASS, mxINT8_CLASS, mxUINT8_CLASS, mxINT16_CLASS, mxUINT16_CLASS,
               mxINT32_CLASS } mxClassID;
typedef int32_t mxInt32;

size_t mxGetM(const mxArray*);
size_t mxGetN(const mxArray*);
size_t mxGetNumberOfElements(const mxArray*);
int mxIsDouble(const mxArray*);
int mxIsInt32(const mxArray*);
int mxIsChar(const mxArray*);
int mxIsCell(const mxArray*);
int mxIsStruct(const mxArray*);
int mxIsClass(const mxArray*, const char*);
double* mxGetDoubles(const mxArray*);
mxInt32* mxGetInt32s(const mxArray*);
double mxGetScalar(const mxArray*);
mxArray* mxGetField(const mxArray*, mwIndex, const char*);
mxArray* mxGetCell(const mxArray*, mwIndex);
char* mxArrayToString(const mxArray*);
mxArray* mxCreateDoubleMatrix(mwSize, mwSize, mxComplexity);
mxArray* mxCreateDoubleScalar(double);
mxArray* mxCreateNumericArray(mwSize, const mwSize*, mxClassID, mxComplexity);
mxArray* mxCreateCellMatrix(mwSize, mwSize);
mxArray* mxCreateString(const char*);
mxArray* mxCreateStructMatrix(mwSize, mwSize, int, const char**);
void mxSetCell(mxArray*, mwIndex, mxArray*);
void mxSetField(mxArray*, mwIndex, const char*, mxArray*);
mxArray* mxDuplicateArray(const mxArray*);
void mxDestroyArray(mxArray*);
void* mxMalloc(size_t);
void* mxCalloc(size_t, size_t);
void mxFree(void*);
void mexErrMsgIdAndTxt(const char*, const char*, ...);
int mexPrintf(const char*, ...);
int mexAtExit(void (*)(void));
int mexCallMATLAB(int, mxArray*[], int, mxArray*[], const char*);
#endif
