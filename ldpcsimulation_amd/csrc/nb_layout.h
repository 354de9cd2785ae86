// nb_layout.h -- constants and message-layout arithmetic of the GF(q) EMS kernels
// shared by the device code (nb.hip) and the host-only graph code (nb_graph.cpp),
// which is also built without HIP for the host sanitizer (Makefile `asan`).
#pragma once

#if defined(__HIPCC__) || defined(__HIP__)
#define LDPC_NB_HD __host__ __device__
#else
#define LDPC_NB_HD
#endif

namespace ldpc {

constexpr int kNbQ = 16;          // field size the kernels are built for (GF(16), BASELINE config 5)
constexpr int kNbMaxDc = 8;       // row degree bound (DC template 4 / 8)

// Position-major message slot count (maxdc * M) rounded up to a power of two
// (at least 4): the chunk stride of the message layout of nb.hip, where the byte
// offset of entry p of slot s is (s << 4) ^ nb_lambda(p) -- XOR-linear in p.
LDPC_NB_HD inline int nb_ep(int maxdc, int M)
{
    int e = 4;
    while (e < maxdc * M) e <<= 1;
    return e;
}
LDPC_NB_HD inline int nb_ep_log2(int ep)
{
    int k = 0;
    while ((1 << k) < ep) ++k;
    return k;
}
// Byte offset of entry p (0..15) relative to its slot's s << 4, chunk stride 2^k slots:
// chunk p >> 2 at (p >> 2) << (k + 4), the slot XOR-ed with the chunk index (bits 4-5),
// the entry within its 16-byte chunk at (p & 3) << 2.
LDPC_NB_HD inline int nb_lambda(int p, int k) { return (p << 2) ^ ((p >> 2) << (k + 4)); }

}  // namespace ldpc
