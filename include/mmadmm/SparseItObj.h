// SparseItObj.h -- the reference's LASolver umbrella header (lib/LASolver/SparseItObj.h: the
// General_Exception utility and the MatrixIter classes), here the MI355X mirror in MatrixIter.h.
#ifndef SPARSEIT_OBJ_INC
#define SPARSEIT_OBJ_INC

#include "MatrixIter.h"

#endif
