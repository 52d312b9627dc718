// NodeType.h -- node types of the reference (src/NodeType.h:4-8), same enumerators and values
// (the C-ABI's MMADMM_BOUNDARY_FREE / MMADMM_BOUNDARY_FIXED / MMADMM_INTERIOR).  Same include
// guard as the reference's header, so a translation unit may include either or both.
#ifndef NODE_TYPE_H
#define NODE_TYPE_H

enum NodeType {
    BOUNDARY_FREE,
    BOUNDARY_FIXED,
    INTERIOR
};

#endif
