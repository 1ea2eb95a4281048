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
//   include/Decoder_Symbol_Wise.h:15-79  | siphon::Decoder_Symbol_Wise (the relay's symbol-wise
//                                        |   decode-and-forward, types 2 and 3), GF work on the GPU
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
    Memory_Allocator(const Memory_Allocator&) = delete;  // owns its buffers / device coder
    Memory_Allocator& operator=(const Memory_Allocator&) = delete;
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
    FEC_Encoder(const FEC_Encoder&) = delete;  // owns its buffers / device coder
    FEC_Encoder& operator=(const FEC_Encoder&) = delete;
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
    FEC_Decoder(const FEC_Decoder&) = delete;  // owns its buffers / device coder
    FEC_Decoder& operator=(const FEC_Decoder&) = delete;
    unsigned char* onReceive(unsigned char* codeword_received, int codeword_size, int seq, int* payload,
                             bool erasure);
    Decoder* decoder;

private:
    Memory_Allocator* memory_object;
    fec_decoder* impl;
    int k, n, T, B, N, max_payload, max_blocklength;
    unsigned char* data_with_header;
};

// ---- relay: Decoder_Symbol_Wise (include/Decoder_Symbol_Wise.h:15-79) --------------------------
// The same public members (the relay and destination code of Variable_Rate_FEC_Decoder writes the
// received packets, erasure flags and headers straight into them, Variable_Rate_FEC_Decoder.cpp
// :1051-1103, :1458-1600, :1703-1870) and methods.  The control flow of every method runs on the
// host over those members (it depends only on flags and headers); its GF work -- the diagonal
// decodes (decodeBlock, T = n-1) and re-encodes (encodeBlock, t = k2-1) of all the packet's code
// blocks -- is one GPU launch per call (fec_sw_* in fec_amd.h).  Differences from the reference,
// all of them its undefined behaviour: the decodes of symbol_wise_encode_1 /
// symbol_wise_decode_1 see the window's n erasure flags (not n-1 plus heap bytes), slots are
// GLOBAL_MAX_SIZE_OF_CODEWORD + 16 bytes (the reference copies that many bytes to offset 2 of a
// slot of that size), temp_codeword's stale bytes are never forwarded; k2 == k is required (as the
// reference assumes, Decoder_Symbol_Wise.cpp:185); FLAG_FOR_SDBO is 0 (FEC_Macro.h:50).
// Slot pointers are not stable: push_current_codeword and rotate_pointers_and_insert_zero_word
// rotate the codeword_vector_state_dependent / header row pointers instead of copying 30 slots of
// contents (Decoder_Symbol_Wise.cpp:131-135, :167-171), so a caller must re-read a slot through the
// member arrays after those calls rather than keep a pointer to it across them (the reference's
// own callers, Variable_Rate_FEC_Decoder.cpp:636-675 and :1458-1493, always index the arrays).
#ifdef T_TOT
static_assert(T_TOT == 10, "the MI355X relay is built for T_TOT = 10 (FEC_Macro.h:32)");
#endif
namespace siphon {
class Decoder_Symbol_Wise {
public:
    static constexpr int kTTot = 10;  // T_TOT
    explicit Decoder_Symbol_Wise(int max_payload_value);
    virtual ~Decoder_Symbol_Wise();
    Decoder_Symbol_Wise(const Decoder_Symbol_Wise&) = delete;  // owns its slot arrays
    Decoder_Symbol_Wise& operator=(const Decoder_Symbol_Wise&) = delete;

    unsigned char* codeword;
    unsigned char** codeword_vector;
    unsigned char** codeword_new_vector;
    unsigned char** codeword_vector_to_transmit;
    unsigned char** codeword_vector_store_in_burst;
    unsigned char** codeword_vector_to_trasnmit_store;

    unsigned char** codeword_vector_state_dependent;
    bool* temp_erasure_vector_state_dependent;
    int** header;

    unsigned char codeword_new_symbol_wise[30000];
    bool* temp_erasure_vector;
    int n2_vector[kTTot + 1];
    int k2_vector[kTTot + 1];

    Decoder* decoder_current;
    Encoder* encoder_current;

    void symbol_wise_encode_1(int k, int n, int k2, int n2, bool* flag);
    void rotate_pointers_and_insert_zero_word(int n, int n2, int temp_size, int codeword_r_d_size_current,
                                              bool flag_fot_rotate_burst);
    void push_current_codeword(unsigned char* message, int n, int n2, int temp_size, int codeword_r_d_size_current);
    void symbol_wise_decode_1(unsigned char* buffer, bool* flag, int k, int n);
    void symbol_wise_encode_state_dependent(int k, int n, int k2, int n2, bool* flag);
    void symbol_wise_decode_state_dependent(unsigned char* buffer, bool* flag, int k, int n);
    void extract_data(unsigned char* buffer, int k, int n, int received_seq, unsigned char* temp_buffer);
    void copy_elements(Decoder_Symbol_Wise* source, bool encode);

    int max_payload;
    int k, n;
    int n2;
    int codeword_size_vector[kTTot + 1];
    int store_codeword_size_vector[kTTot + 1];
    int burst_codeword_size_vector[kTTot + 1];

private:
    void shift(int n, int n2);
};
}  // namespace siphon

