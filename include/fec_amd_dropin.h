// fec_amd_dropin.h -- the reference's C++ API for the coding path, re-implemented over the
// MI355X C ABI (fec_amd.h) so that Variable_Rate_FEC_Encoder / Variable_Rate_FEC_Decoder /
// Application_Layer_Sender / Application_Layer_Receiver compile against it (tests/test_dropin_compile.py).
//
//   reference header                     | here
//   include/Memory_Allocator.h:17-31     | Memory_Allocator (ring of 33000-byte buffers)
//   include/FEC_Message.h:17-31          | FEC_Message (plain carrier)
//   include/FEC_Encoder.h:26-48          | FEC_Encoder(max_payload,T,B,N,Memory_Allocator*),
//                                        |   onTransmit(data,payload,seq,&codeword_size)
//   include/FEC_Decoder.h:27-46          | FEC_Decoder(max_payload,T,B,N,Memory_Allocator*),
//                                        |   onReceive(codeword,codeword_size,seq,&payload,erasure)
//   include/Encoder.h / Decoder.h getG() | Encoder::getG(), Decoder::getG() (public members
//                                        |   FEC_Encoder::encoder / FEC_Decoder::decoder)
//
// Semantics kept: one call per seq in increasing order from 0; onTransmit returns a pointer into
// the caller's Memory_Allocator ring (two allocations per call, like FEC_Encoder.cpp:48,62);
// onReceive copies the wire codeword into one ring buffer (FEC_Decoder.cpp:55) and returns a
// pointer to the decoder's own buffer, valid until the next call; *payload = 0 means lost / not
// yet available.  Construction failures (no HIP device, unsupported (T,B,N)) throw
// std::runtime_error -- the reference has no error channel at all.
#pragma once

// The transitive surface of the six reference headers this one replaces (FEC_Encoder.h:17-24,
// FEC_Decoder.h:17-25, Memory_Allocator.h:17, Encoder.h -> Encoder_Basic.h -> ... ): their callers
// (Variable_Rate_FEC_Encoder.cpp, Variable_Rate_FEC_Decoder.cpp, Decoder_Symbol_Wise.cpp,
// Application_Layer_Sender/Receiver.cpp) use std::string, std::ofstream, ceil, memcpy and the
// <random> engines without including them.  tests/test_dropin_compile.py compiles those callers
// against this header.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <random>
#include <string>

using std::string;
using std::ofstream;

struct fec_encoder;
struct fec_decoder;
struct fec_codec;

class Memory_Allocator {
public:
    explicit Memory_Allocator(int number_of_buffers);
    virtual ~Memory_Allocator();
    unsigned char* allocate_memory(int size);

private:
    unsigned char** buffer;
    int unallocated_buffer_index;
    int number_of_buffers;
};

class FEC_Message {
public:
    FEC_Message();
    void set_parameters(int seq_number_value, int T_value, int B_value, int N_value, int size_value,
                        unsigned char* buffer_ptr);
    virtual ~FEC_Message();
    int seq_number, T, B, N, counter_for_start_and_end, size;
    int seq_number2;
    unsigned char* buffer;
};

class Encoder {
public:
    Encoder(int T_value, int B_value, int N_value, int max_payload_value);
    virtual ~Encoder();
    unsigned char* getG();
    int T, B, N, max_payload;

private:
    unsigned char* G;
};

class Decoder {
public:
    Decoder(int T_value, int B_value, int N_value, int max_payload_value);
    virtual ~Decoder();
    unsigned char* getG();
    int T, B, N, max_payload;

private:
    unsigned char* G;
};

class FEC_Encoder {
public:
    FEC_Encoder(int max_payload_value, int T_value, int B_value, int N_value, Memory_Allocator* memory);
    virtual ~FEC_Encoder();
    unsigned char* onTransmit(unsigned char* data, int payload, int seq, int* codeword_size);
    Encoder* encoder;

private:
    Memory_Allocator* memory_object;
    fec_encoder* impl;
    int T, B, N, k, n, max_payload, max_blocklength;
};

class FEC_Decoder {
public:
    FEC_Decoder(int max_payload_value, int T_value, int B_value, int N_value, Memory_Allocator* memory);
    virtual ~FEC_Decoder();
    unsigned char* onReceive(unsigned char* codeword_received, int codeword_size, int seq, int* payload,
                             bool erasure);
    Decoder* decoder;

private:
    Memory_Allocator* memory_object;
    fec_decoder* impl;
    int k, n, T, B, N, max_payload, max_blocklength;
    unsigned char* data_with_header;
};
