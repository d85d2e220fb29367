// rs16_comm.cpp -- RCCL over xGMI for the multi-GPU configuration (SURVEY.md
// 8(e), BASELINE configs[4]): a stripe that lives in one GPU's HBM is split
// into byte-column slices, one per rank, and the slices are brought back
// after every rank has run the codec on its own.  Every 64-byte column block
// is an independent codeword (src/algorithm.md:18-32), so the codec itself
// needs no exchange; the scatter and the gather are the only collectives.
//
// A column slice of a row-major stripe is strided (width w of every S-byte
// row), and RCCL moves contiguous buffers: the root packs the slices with one
// pitched device copy each into a staging buffer (rank r's slice = rows x w_r
// contiguous bytes = a shard array of shard_bytes w_r), then one grouped
// ncclSend / ncclRecv per rank moves them over xGMI.  The gather is the
// mirror image.  The root's own slice never enters RCCL: one pitched device
// copy between its full array and its slice.  Ranks may be processes (one rs16_comm each, ncclCommInitRank
// with a shared unique id) or engines of one process (rs16_comm_init_all,
// ncclCommInitAll); the collective calls take the array of this process's
// communicators and issue them in one NCCL group.
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "rs16_engine.hpp"

using namespace rs16;

struct rs16_comm {
    rs16_engine* eng = nullptr;
    ncclComm_t nc = nullptr;
    int nranks = 0, rank = 0;
    bool blocking = false;  // ncclCommInitAll communicators are blocking
    DevBuf stage;  // root: packed column slices
};

static int nccl_fail(rs16_error* err, ncclResult_t r) { return set_error(err, RS16_DEVICE_ERROR, 1000 + (uint64_t)r); }
#define RS16_NCCL(call)                                     \
    do {                                                    \
        ncclResult_t _r = (call);                           \
        if (_r != ncclSuccess) return nccl_fail(err, _r);   \
    } while (0)

// Communicators are non-blocking (ncclConfig_t::blocking = 0): init and
// every group of sends / receives return at once and are waited for here
// with a deadline, so a rank that never joins makes the others fail with an
// error (the communicator aborted) instead of hanging the process.
static constexpr double INIT_DEADLINE_S = 120.0, GROUP_DEADLINE_S = 60.0;
static ncclResult_t settle(ncclComm_t c, ncclResult_t r, double deadline_s) {
    if (r != ncclSuccess && r != ncclInProgress) return r;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        ncclResult_t q = ncclCommGetAsyncError(c, &st);
        if (q != ncclSuccess) return q;
        if (st != ncclInProgress) return st;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > deadline_s) {
            (void)ncclCommAbort(c);
            return ncclSystemError;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Column slice of rank r of n (B = S / 64 blocks).
static void col_slice(size_t S, int n, int r, size_t* off, size_t* w) {
    // whole 64-byte blocks, the first (B mod n) slices one block wider (rs16/columns.py)
    const size_t blocks = S / 64, base = blocks / (size_t)n, extra = blocks % (size_t)n, x = (size_t)r;
    *off = (x * base + (x < extra ? x : extra)) * 64;
    *w = (base + (x < extra ? 1 : 0)) * 64;
}

extern "C" int rs16_comm_unique_id(void* id, rs16_error* err) {
    if (!id) return set_error(err, RS16_INVALID_ARGUMENT);
    ncclUniqueId u;
    RS16_NCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return set_error(err, RS16_OK);
}

extern "C" rs16_comm* rs16_comm_new(rs16_engine* eng, int nranks, int rank, const void* id, rs16_error* err) {
    if (!eng || !id || nranks < 1 || rank < 0 || rank >= nranks) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    if (eng->activate(err)) return nullptr;
    rs16_comm* c = new (std::nothrow) rs16_comm();
    if (!c) return set_error(err, RS16_INVALID_ARGUMENT), nullptr;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c->nc, nranks, u, rank, &cfg);
    if (c->nc) r = settle(c->nc, r, INIT_DEADLINE_S);
    if (r != ncclSuccess) {
        c->nc = nullptr;  // (aborted, or never created)
        delete c;
        return nccl_fail(err, r), nullptr;
    }
    c->eng = eng;
    c->nranks = nranks;
    c->rank = rank;
    set_error(err, RS16_OK);
    return c;
}

extern "C" int rs16_comm_init_all(rs16_engine* const* engines, int n, rs16_comm** comms, rs16_error* err) {
    if (!engines || !comms || n < 1) return set_error(err, RS16_INVALID_ARGUMENT);
    std::vector<int> devs(n);
    for (int i = 0; i < n; i++) {
        if (!engines[i]) return set_error(err, RS16_INVALID_ARGUMENT);
        devs[i] = engines[i]->device;
    }
    std::vector<ncclComm_t> nc(n);
    RS16_NCCL(ncclCommInitAll(nc.data(), n, devs.data()));
    for (int i = 0; i < n; i++) {
        comms[i] = new (std::nothrow) rs16_comm();
        if (!comms[i]) return set_error(err, RS16_INVALID_ARGUMENT);
        comms[i]->eng = engines[i];
        comms[i]->nc = nc[i];
        comms[i]->nranks = n;
        comms[i]->rank = i;
        comms[i]->blocking = true;
    }
    return set_error(err, RS16_OK);
}

extern "C" void rs16_comm_free(rs16_comm* c) {
    if (!c) return;
    if (c->eng) {
        (void)hipSetDevice(c->eng->device);
        (void)hipStreamSynchronize(c->eng->stream);
    }
    if (c->nc) (void)ncclCommDestroy(c->nc);
    c->stage.release();
    delete c;
}

extern "C" int rs16_comm_rank(const rs16_comm* c) { return c->rank; }
extern "C" int rs16_comm_size(const rs16_comm* c) { return c->nranks; }
extern "C" int rs16_column_slice(size_t shard_bytes, int nranks, int rank, size_t* offset, size_t* width) {
    if (nranks < 1 || rank < 0 || rank >= nranks || shard_bytes % 64) return RS16_INVALID_ARGUMENT;
    col_slice(shard_bytes, nranks, rank, offset, width);
    return RS16_OK;
}

// The root's rows x S array <-> every rank's rows x w_r column slice.
// d_full[i] / d_slice[i] belong to comms[i] (d_full only read / written on the root).
static int columns(rs16_comm* const* comms, int n, int root, size_t rows, size_t S, void* const* d_full,
                   void* const* d_slice, void* stream, bool scatter, rs16_error* err) {
    if (!comms || n < 1 || (S % 64) || S == 0) return set_error(err, RS16_INVALID_ARGUMENT);
    const int nranks = comms[0]->nranks;
    if (root < 0 || root >= nranks) return set_error(err, RS16_INVALID_ARGUMENT);
    for (int i = 0; i < n; i++)
        if (!comms[i] || !comms[i]->nc || comms[i]->nranks != nranks) return set_error(err, RS16_INVALID_ARGUMENT);
    auto strm = [&](rs16_comm* c) { return (n == 1 && stream) ? (hipStream_t)stream : c->eng->stream; };
    // root: its own slice directly; scatter: pack the other ranks' slices
    // (one pitched copy per rank)
    for (int i = 0; i < n; i++) {
        rs16_comm* c = comms[i];
        if (c->rank != root) continue;
        if (int rc = c->eng->activate(err)) return rc;
        size_t off, w;
        col_slice(S, nranks, root, &off, &w);
        if (w && scatter)
            RS16_HIP(hipMemcpy2DAsync(d_slice[i], w, (const uint8_t*)d_full[i] + off, S, w, rows,
                                      hipMemcpyDeviceToDevice, strm(c)));
        if (w && !scatter)
            RS16_HIP(hipMemcpy2DAsync((uint8_t*)d_full[i] + off, S, d_slice[i], w, w, rows, hipMemcpyDeviceToDevice,
                                      strm(c)));
        if (nranks == 1) continue;
        RS16_HIP(c->stage.reserve(rows * S));
        if (scatter)
            for (int r = 0; r < nranks; r++) {
                col_slice(S, nranks, r, &off, &w);
                if (!w || r == root) continue;
                RS16_HIP(hipMemcpy2DAsync((uint8_t*)c->stage.p + rows * off, w, (const uint8_t*)d_full[i] + off, S, w,
                                          rows, hipMemcpyDeviceToDevice, strm(c)));
            }
    }
    if (nranks == 1) return set_error(err, RS16_OK);
    RS16_NCCL(ncclGroupStart());
    for (int i = 0; i < n; i++) {
        rs16_comm* c = comms[i];
        if (int rc = c->eng->activate(err)) {
            (void)ncclGroupEnd();
            return rc;
        }
        size_t off, w;
        col_slice(S, nranks, c->rank, &off, &w);
        if (c->rank == root) {
            for (int r = 0; r < nranks; r++) {
                size_t o2, w2;
                col_slice(S, nranks, r, &o2, &w2);
                if (!w2 || r == root) continue;
                uint8_t* p = (uint8_t*)c->stage.p + rows * o2;
                ncclResult_t x = scatter ? ncclSend(p, rows * w2, ncclUint8, r, c->nc, strm(c))
                                         : ncclRecv(p, rows * w2, ncclUint8, r, c->nc, strm(c));
                if (x != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return nccl_fail(err, x);
                }
            }
        }
        if (w && c->rank != root) {
            ncclResult_t x = scatter ? ncclRecv(d_slice[i], rows * w, ncclUint8, root, c->nc, strm(c))
                                     : ncclSend(d_slice[i], rows * w, ncclUint8, root, c->nc, strm(c));
            if (x != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_fail(err, x);
            }
        }
    }
    {
        const ncclResult_t g = ncclGroupEnd();
        for (int i = 0; i < n; i++) {
            const ncclResult_t x = comms[i]->blocking ? g : settle(comms[i]->nc, g, GROUP_DEADLINE_S);
            if (x != ncclSuccess) {
                if (!comms[i]->blocking) comms[i]->nc = nullptr;  // (aborted by settle)
                return nccl_fail(err, x);
            }
        }
    }
    // root, gather: unpack into the full rows x S array
    if (!scatter)
        for (int i = 0; i < n; i++) {
            rs16_comm* c = comms[i];
            if (c->rank != root) continue;
            if (int rc = c->eng->activate(err)) return rc;
            for (int r = 0; r < nranks; r++) {
                size_t off, w;
                col_slice(S, nranks, r, &off, &w);
                if (!w || r == root) continue;
                RS16_HIP(hipMemcpy2DAsync((uint8_t*)d_full[i] + off, S, (const uint8_t*)c->stage.p + rows * off, w, w,
                                          rows, hipMemcpyDeviceToDevice, strm(c)));
            }
        }
    return set_error(err, RS16_OK);
}

extern "C" int rs16_scatter_columns(rs16_comm* const* comms, int n, int root, size_t rows, size_t shard_bytes,
                                    const void* const* d_full, void* const* d_slice, void* stream, rs16_error* err) {
    return columns(comms, n, root, rows, shard_bytes, (void* const*)d_full, d_slice, stream, true, err);
}
extern "C" int rs16_gather_columns(rs16_comm* const* comms, int n, int root, size_t rows, size_t shard_bytes,
                                   const void* const* d_slice, void* const* d_full, void* stream, rs16_error* err) {
    return columns(comms, n, root, rows, shard_bytes, d_full, (void* const*)d_slice, stream, false, err);
}
