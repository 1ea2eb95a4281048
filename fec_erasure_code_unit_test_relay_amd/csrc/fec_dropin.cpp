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

// ---- Decoder_Symbol_Wise (src/Decoder_Symbol_Wise.cpp:16-665) -------------------------------
namespace siphon {
namespace {
constexpr int kTT = Decoder_Symbol_Wise::kTTot;
constexpr int kGlobalMax = 20000;           // GLOBAL_MAX_SIZE_OF_CODEWORD (FEC_Macro.h:49)
constexpr int kSlot = kGlobalMax + 16;      // the reference writes kGlobalMax bytes at offset 2
static_assert(sizeof(bool) == 1, "flag arrays are handed to the C ABI as bytes");
unsigned char** slots(int count) {
    unsigned char** v = static_cast<unsigned char**>(std::calloc(count, sizeof(unsigned char*)));
    for (int i = 0; i < count; ++i) v[i] = static_cast<unsigned char*>(std::calloc(kSlot, 1));
    return v;
}
void free_slots(unsigned char** v, int count) {
    if (!v) return;
    for (int i = 0; i < count; ++i) std::free(v[i]);
    std::free(v);
}
void check_sw(const char* what, int st) {
    if (st) fail(what, st);
}
}  // namespace

// :16-65
Decoder_Symbol_Wise::Decoder_Symbol_Wise(int max_payload_value)
    : codeword(nullptr), decoder_current(nullptr), encoder_current(nullptr), max_payload(max_payload_value), k(0),
      n(0), n2(0) {
    codeword_vector = slots(kTT + 1);
    codeword_new_vector = slots(kTT + 1);
    codeword_vector_store_in_burst = slots(kTT + 1);
    codeword_vector_to_transmit = slots(kTT + 1);
    codeword_vector_to_trasnmit_store = slots(kTT + 1);
    temp_erasure_vector = static_cast<bool*>(std::calloc(kTT + 1, sizeof(bool)));
    codeword_vector_state_dependent = slots(3 * kTT);
    temp_erasure_vector_state_dependent = static_cast<bool*>(std::calloc(3 * kTT, sizeof(bool)));
    header = static_cast<int**>(std::calloc(3 * kTT, sizeof(int*)));
    for (int i = 0; i < 3 * kTT; ++i) {
        header[i] = static_cast<int*>(std::calloc(kTT + 1, sizeof(int)));
        for (int jj = 0; jj < kTT + 1; ++jj) header[i][jj] = jj + 1;
    }
    for (int i = 0; i < kTT + 1; ++i) {
        n2_vector[i] = k2_vector[i] = 0;
        codeword_size_vector[i] = store_codeword_size_vector[i] = burst_codeword_size_vector[i] = 0;
    }
    std::memset(codeword_new_symbol_wise, 0, sizeof(codeword_new_symbol_wise));
}

// :67-86 (the encoder is freed too: copy_elements always gives each object its own)
Decoder_Symbol_Wise::~Decoder_Symbol_Wise() {
    free_slots(codeword_vector, kTT + 1);
    free_slots(codeword_new_vector, kTT + 1);
    free_slots(codeword_vector_store_in_burst, kTT + 1);
    free_slots(codeword_vector_to_transmit, kTT + 1);
    free_slots(codeword_vector_to_trasnmit_store, kTT + 1);
    free_slots(codeword_vector_state_dependent, 3 * kTT);
    for (int i = 0; i < 3 * kTT; ++i) std::free(header[i]);
    std::free(header);
    std::free(temp_erasure_vector_state_dependent);
    std::free(temp_erasure_vector);
    delete decoder_current;
    delete encoder_current;
}

// :88-117
void Decoder_Symbol_Wise::copy_elements(Decoder_Symbol_Wise* source, bool encode) {
    for (int i = 0; i < kTT + 1; ++i) {
        std::memcpy(codeword_vector[i], source->codeword_vector[i], kGlobalMax);
        std::memcpy(codeword_new_vector[i], source->codeword_new_vector[i], kGlobalMax);
        std::memcpy(codeword_vector_store_in_burst[i], source->codeword_vector_store_in_burst[i], kGlobalMax);
        std::memcpy(codeword_vector_to_transmit[i], source->codeword_vector_to_transmit[i], kGlobalMax);
        temp_erasure_vector[i] = source->temp_erasure_vector[i];
        burst_codeword_size_vector[i] = source->burst_codeword_size_vector[i];
        codeword_size_vector[i] = source->codeword_size_vector[i];
    }
    for (int i = 0; i < 3 * kTT; ++i) {
        std::memcpy(codeword_vector_state_dependent[i], source->codeword_vector_state_dependent[i], kGlobalMax);
        std::memcpy(header[i], source->header[i], sizeof(int) * (kTT + 1));
        temp_erasure_vector_state_dependent[i] = source->temp_erasure_vector_state_dependent[i];
    }
    delete decoder_current;
    decoder_current = new Decoder(source->decoder_current->T, source->decoder_current->B, source->decoder_current->N,
                                  source->decoder_current->max_payload);
    if (encode) {
        delete encoder_current;
        encoder_current = new Encoder(source->encoder_current->T, source->encoder_current->B,
                                      source->encoder_current->N, source->encoder_current->max_payload);
    }
}

// the shifts common to push_current_codeword (:119-135) and rotate_pointers_and_insert_zero_word
// (:142-171): contents move down one slot, the top slot keeps its own; header rows move their
// first T_TOT ints (entry T_TOT of a row stays, :133, :169)
void Decoder_Symbol_Wise::shift(int nn, int nn2) {
    for (int i = 0; i < nn - 1; ++i) {
        std::memcpy(codeword_vector[i], codeword_vector[i + 1], kGlobalMax);
        temp_erasure_vector[i] = temp_erasure_vector[i + 1];
    }
    for (int i = 0; i < nn2 - 1; ++i) {
        std::memcpy(codeword_new_vector[i], codeword_new_vector[i + 1], kGlobalMax);
        std::memcpy(codeword_vector_to_transmit[i], codeword_vector_to_transmit[i + 1], kGlobalMax);
        codeword_size_vector[i] = codeword_size_vector[i + 1];
        k2_vector[i] = k2_vector[i + 1];
    }
    // the state-dependent slots by pointer: the slot that falls off the bottom becomes the top one
    // with the top one's content (what the reference's copies leave there)
    unsigned char* bottom = codeword_vector_state_dependent[0];
    for (int i = 0; i < 3 * kTT - 1; ++i) {
        codeword_vector_state_dependent[i] = codeword_vector_state_dependent[i + 1];
        std::memcpy(header[i], header[i + 1], sizeof(int) * kTT);
        temp_erasure_vector_state_dependent[i] = temp_erasure_vector_state_dependent[i + 1];
    }
    std::memcpy(bottom, codeword_vector_state_dependent[3 * kTT - 2], kSlot);
    codeword_vector_state_dependent[3 * kTT - 1] = bottom;
}

// :119-140 (the message is copied with GLOBAL_MAX_SIZE_OF_CODEWORD bytes, as the reference does)
void Decoder_Symbol_Wise::push_current_codeword(unsigned char* message, int nn, int nn2, int, int) {
    shift(nn, nn2);
    std::memcpy(&codeword_vector[nn - 1][2], message, kGlobalMax);
    temp_erasure_vector[nn - 1] = false;
}

// :142-176
void Decoder_Symbol_Wise::rotate_pointers_and_insert_zero_word(int nn, int nn2, int, int, bool flag_burst) {
    if (flag_burst)
        for (int i = 0; i < nn - 1; ++i) {
            std::memcpy(codeword_vector_store_in_burst[i], codeword_vector_store_in_burst[i + 1], kGlobalMax);
            burst_codeword_size_vector[i] = burst_codeword_size_vector[i + 1];
        }
    shift(nn, nn2);
    std::memset(codeword_vector[nn - 1], 0, kGlobalMax);
    temp_erasure_vector[nn - 1] = true;
}

// :178-432
void Decoder_Symbol_Wise::symbol_wise_encode_state_dependent(int kk, int nn, int kk2, int nn2, bool* flag) {
    *flag = false;  // :195, never set
    check_sw("symbol_wise_encode_state_dependent",
             fec_sw_state_encode(max_payload, kk, nn, kk2, nn2, 0, codeword_vector_state_dependent,
                                 reinterpret_cast<const uint8_t*>(temp_erasure_vector_state_dependent), header,
                                 codeword_new_vector[nn2 - 1], codeword_new_symbol_wise));
}

// :487-546
void Decoder_Symbol_Wise::symbol_wise_decode_state_dependent(unsigned char* buffer, bool* flag, int kk, int nn) {
    int fl = 0;
    check_sw("symbol_wise_decode_state_dependent",
             fec_sw_state_decode(max_payload, kk, nn, codeword_vector_state_dependent, header, buffer, &fl));
    *flag = fl != 0;
}

// :547-619
void Decoder_Symbol_Wise::symbol_wise_encode_1(int kk, int nn, int kk2, int nn2, bool* flag) {
    int fl = 0;
    check_sw("symbol_wise_encode_1",
             fec_sw_encode_1(max_payload, kk, nn, kk2, nn2, codeword_vector,
                             reinterpret_cast<const uint8_t*>(temp_erasure_vector), codeword_new_vector,
                             codeword_new_symbol_wise, &fl));
    *flag = fl != 0;
}

// :621-651
void Decoder_Symbol_Wise::symbol_wise_decode_1(unsigned char* buffer, bool* flag, int kk, int nn) {
    int fl = 0;
    check_sw("symbol_wise_decode_1",
             fec_sw_decode_1(max_payload, kk, nn, codeword_vector, reinterpret_cast<const uint8_t*>(temp_erasure_vector),
                             buffer, &fl));
    *flag = fl != 0;
}

// :653-665 (a copy, no GF work; the debug print is not reproduced)
void Decoder_Symbol_Wise::extract_data(unsigned char* buffer, int kk, int nn, int, unsigned char* temp_buffer) {
    const int blocks = max_payload / kk + 1;
    int ind = 0;
    for (int j = 0; j < blocks; ++j)
        for (int i = 0; i < kk; ++i) temp_buffer[ind++] = buffer[j * nn + nn - kk + i];
}
}  // namespace siphon
