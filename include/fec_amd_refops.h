// fec_amd_refops.h -- the reference's free GF(2^8) and block-code functions with their own
// signatures, defined by libfec_amd.so over the library's host field (fec_host.h), so that a
// reference build under the header swap needs neither basicOperations.cpp,
// codingOperations.cpp nor Intel ISA-L.
//
//   reference declaration                          | here
//   include/basicOperations.h:6-24                 | gf256_add / _mul / _inv / _invert_matrix /
//                                                  |   _rref_matrix / _transpose / _matrix_mul,
//                                                  |   printMatrix (both overloads)
//   include/codingOperations.h:27-41               | init_at_sender, encodeBlock, decodeBlock,
//                                                  |   generateData, gen_G_cauchy, save_to_file,
//                                                  |   calculateLoss, calculateLossMessage
//
// The two reference headers become forwarders to this one (basicOperations.h keeps its
// FEC_Macro.h include); this header carries codingOperations.h's transitive surface (<cstdlib>
// <iostream> <sstream> <fstream>, using std::cout / endl / string / ofstream).
// Semantics: the reference's (basicOperations.cpp:14-202, codingOperations.cpp:27-297), with
// ISA-L's field (poly 0x11d, generator 2) and ISA-L's gf_invert_matrix / gf_gen_cauchy1_matrix /
// gf_gen_rs_matrix restated; the one deliberate difference is that the unsigned-char
// printMatrix prints only when the including translation unit has DEBUG_FEC == 1 (the reference
// compiled that test into basicOperations.cpp, FEC_Macro.h:107 sets it to 0).
#pragma once

#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

using std::cout;
using std::endl;
using std::ofstream;
using std::string;

unsigned char gf256_add(unsigned char a, unsigned char b);
unsigned char gf256_mul(unsigned char a, unsigned char b);
unsigned char gf256_inv(unsigned char a);
int gf256_invert_matrix(unsigned char *in, unsigned char *out, const int n);
void gf256_rref_matrix(unsigned char *in, unsigned char *out, unsigned char *action, int k, int n);
void gf256_transpose(unsigned char *in, unsigned char *out, int k, int n);
void gf256_matrix_mul(unsigned char *inMatrix1, unsigned char *inMatrix2, unsigned char *outMatrix, int m1, int m2,
                      int m3);
void printMatrix(bool *matrix, int row, int column);
void fec_print_matrix_u8(const unsigned char *matrix, int row, int column);  // printMatrix's body, unconditional
inline void printMatrix(unsigned char *matrix, int row, int column) {
#if defined(DEBUG_FEC) && DEBUG_FEC == 1
    fec_print_matrix_u8(matrix, row, column);
#else
    (void)matrix;
    (void)row;
    (void)column;
#endif
}

int init_at_sender(int T, int B, int N, unsigned char *G, int k, int n);
void encodeBlock(unsigned char *data, unsigned char *generator, unsigned char *codeword, int k, int n, int t);
void decodeBlock(unsigned char *data, unsigned char *generator, unsigned char *codeword, bool *erasure, int k, int n,
                 int T, int t);
void generateData(unsigned char *data, int k);
void gen_G_cauchy(unsigned char *G, int T, int B, int N, int k, int n);
void save_to_file(unsigned char *data, int payload, ofstream *file);
float calculateLoss(unsigned char *data, unsigned char *recovered_data, int max_payload, int *payload,
                    int stream_duration, int T);
float calculateLossMessage(string file_original, string file_recovered);
