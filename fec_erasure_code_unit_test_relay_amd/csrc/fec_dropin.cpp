// fec_dropin.cpp -- the reference's C++ coding API (include/fec_amd_dropin.h) over the C ABI.
#include "fec_amd_dropin.h"

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>

#include "fec_amd.h"
#include "fec_host.h"

namespace {
[[noreturn]] void fail(const char* what, int st) {
    throw std::runtime_error(std::string(what) + ": " + fec_strerror(st));
}
}  // namespace

// ---- Memory_Allocator (src/Memory_Allocator.cpp:20-55) -------------------------------------
Memory_Allocator::Memory_Allocator(int number_of_buffers_value)
    : buffer(nullptr), unallocated_buffer_index(0), number_of_buffers(number_of_buffers_value) {
    buffer = static_cast<unsigned char**>(std::calloc(number_of_buffers, sizeof(unsigned char*)));
    for (int i = 0; i < number_of_buffers; ++i)
        buffer[i] = static_cast<unsigned char*>(std::calloc(33000, 1));
}

Memory_Allocator::~Memory_Allocator() {
    for (int i = 0; i < number_of_buffers; ++i) std::free(buffer[i]);
    std::free(buffer);
}

unsigned char* Memory_Allocator::allocate_memory(int size) {
    if (size > 33000) std::cout << "Cannot allocate memory of size " << size << std::endl;
    if (size <= 0) return nullptr;
    unsigned char* p = buffer[unallocated_buffer_index];
    unallocated_buffer_index = (unallocated_buffer_index + 1) % number_of_buffers;
    return p;
}

// ---- FEC_Message (src/FEC_Message.cpp:21-42) ------------------------------------------------
FEC_Message::FEC_Message()
    : seq_number(0), T(0), B(0), N(0), counter_for_start_and_end(0), size(0), seq_number2(0),
      buffer(nullptr) {}

void FEC_Message::set_parameters(int s, int t, int b, int nn, int sz, unsigned char* p) {
    seq_number = s;
    size = sz;
    T = t;
    B = b;
    N = nn;
    buffer = p;
}

FEC_Message::~FEC_Message() {}

// ---- Encoder / Decoder: only getG() is reachable from the coding path's callers -------------
Encoder::Encoder(int t, int b, int nn, int mp) : T(t), B(b), N(nn), max_payload(mp), G(nullptr) {
    const auto g = fec::make_generator(t, b, nn);
    G = static_cast<unsigned char*>(std::malloc(g.size()));
    std::memcpy(G, g.data(), g.size());
}
Encoder::~Encoder() { std::free(G); }
unsigned char* Encoder::getG() { return G; }

Decoder::Decoder(int t, int b, int nn, int mp) : T(t), B(b), N(nn), max_payload(mp), G(nullptr) {
    const auto g = fec::make_generator(t, b, nn);
    G = static_cast<unsigned char*>(std::malloc(g.size()));
    std::memcpy(G, g.data(), g.size());
}
Decoder::~Decoder() { std::free(G); }
unsigned char* Decoder::getG() { return G; }

// ---- FEC_Encoder (src/FEC_Encoder.cpp:22-68) ------------------------------------------------
FEC_Encoder::FEC_Encoder(int mp, int t, int b, int nn, Memory_Allocator* memory)
    : encoder(nullptr), memory_object(memory), impl(nullptr), T(t), B(b), N(nn), max_payload(mp) {
    k = T - N + 1;
    n = k + B;
    max_blocklength = ((max_payload + 2 + k - 1) / k) * n;
    if (int st = fec_encoder_create(mp, t, b, nn, &impl)) fail("FEC_Encoder", st);
    encoder = new Encoder(t, b, nn, mp);
}

FEC_Encoder::~FEC_Encoder() {
    delete encoder;
    fec_encoder_destroy(impl);
}

unsigned char* FEC_Encoder::onTransmit(unsigned char* data, int payload, int seq, int* codeword_size) {
    unsigned char* internal = memory_object->allocate_memory(max_blocklength);
    int size = 0;
    if (int st = fec_encoder_transmit(impl, data, payload, seq, internal, &size)) fail("onTransmit", st);
    *codeword_size = size;
    unsigned char* wire = memory_object->allocate_memory(size);
    if (wire && size > 0) std::memcpy(wire, internal, static_cast<size_t>(size));
    return wire;
}

// ---- FEC_Decoder (src/FEC_Decoder.cpp:26-72) ------------------------------------------------
FEC_Decoder::FEC_Decoder(int mp, int t, int b, int nn, Memory_Allocator* memory)
    : decoder(nullptr), memory_object(memory), impl(nullptr), T(t), B(b), N(nn), max_payload(mp) {
    k = T - N + 1;
    n = k + B;
    max_blocklength = ((max_payload + 2 + k - 1) / k) * n;
    if (int st = fec_decoder_create(mp, t, b, nn, &impl)) fail("FEC_Decoder", st);
    decoder = new Decoder(t, b, nn, mp);
    data_with_header = static_cast<unsigned char*>(std::calloc(max_blocklength * k / n + 2, 1));
}

FEC_Decoder::~FEC_Decoder() {
    std::free(data_with_header);
    delete decoder;
    fec_decoder_destroy(impl);
}

unsigned char* FEC_Decoder::onReceive(unsigned char* codeword_input, int codeword_size, int seq,
                                      int* payload, bool erasure) {
    const bool er = erasure || codeword_input == nullptr;
    if (!er) {  // the reference keeps a zero-padded copy in the caller's ring (FEC_Decoder.cpp:55)
        unsigned char* copy = memory_object->allocate_memory(max_blocklength);
        std::memcpy(copy, codeword_input, static_cast<size_t>(codeword_size));
        std::memset(copy + codeword_size, 0, static_cast<size_t>(max_blocklength - codeword_size));
        codeword_input = copy;
    }
    int p = 0;
    if (int st = fec_decoder_receive(impl, er ? nullptr : codeword_input, er ? 0 : codeword_size, seq,
                                     er ? 1 : 0, data_with_header + 2, &p))
        fail("onReceive", st);
    *payload = p;
    return data_with_header + 2;
}
