#define H3T_QUAL static
#include "h3_oracle.c"  /* build with -I oracle */
void ex_set(int f, int i, int j, int k, int v) { H3T_FACE_IJK_BASE_CELLS[f][i][j][k] = (unsigned short)v; }
int ex_get(int f, int i, int j, int k) { return H3T_FACE_IJK_BASE_CELLS[f][i][j][k]; }
