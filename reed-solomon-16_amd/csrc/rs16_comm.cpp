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
    // the last collective's use of `stage` (recorded on its stream): the
    // next collective, on whatever stream, waits for it before repacking
    hipEvent_t stage_ev = nullptr;
    bool stage_busy = false;
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
// On any failure the communicator is aborted here (and must not be used or
// destroyed again by the caller).
static ncclResult_t settle(ncclComm_t c, ncclResult_t r, double deadline_s) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress || r == ncclSuccess) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(c, &st);
        if (q != ncclSuccess) {
            r = q;
            break;
        }
        if (st != ncclInProgress) {
            r = st;
            break;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > deadline_s) {
            r = ncclSystemError;
            break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (r != ncclSuccess) (void)ncclCommAbort(c);
    return r;
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
    if (c->nc) r = settle(c->nc, r, INIT_DEADLINE_S);  // (aborts c->nc on failure)
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
        if (!comms[i]) {
            // nothing half-made survives: every communicator destroyed, every object freed
            for (int j = 0; j < n; j++) (void)ncclCommDestroy(nc[j]);
            for (int j = 0; j < i; j++) delete comms[j], comms[j] = nullptr;
            return set_error(err, RS16_INVALID_ARGUMENT);
        }
    }
    for (int i = 0; i < n; i++) {
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
        // (a collective on a caller's stream: its last use of the staging buffer)
        if (c->stage_busy) (void)hipEventSynchronize(c->stage_ev);
    }
    if (c->nc) (void)ncclCommDestroy(c->nc);
    if (c->stage_ev) (void)hipEventDestroy(c->stage_ev);
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

// The root's rows x S array <-> P column slices, slice j owned by rank
// owner(j).  Normally P = nranks and slice j belongs to rank j; d_full[i] /
// d_slice[i] belong to comms[i] (d_full only read / written on the root).
// Diagnostic virtual slices (vslices = P > 0, a one-rank communicator): all P
// slices are owned by rank 0 itself, d_slice[j] is slice j's buffer, and
// every slice but slice 0 goes through the same staging pack, grouped
// ncclSend / ncclRecv (to the rank itself) and unpack as another rank's slice
// would -- so the multi-rank data path runs on a one-GPU machine
// (tests/test_gpu_rccl.py).
static int columns(rs16_comm* const* comms, int n, int root, size_t rows, size_t S, void* const* d_full,
                   void* const* d_slice, void* stream, bool scatter, rs16_error* err, int vslices = 0) {
    if (!comms || n < 1 || (S % 64) || S == 0) return set_error(err, RS16_INVALID_ARGUMENT);
    const int nranks = comms[0]->nranks;
    if (root < 0 || root >= nranks) return set_error(err, RS16_INVALID_ARGUMENT);
    for (int i = 0; i < n; i++)
        if (!comms[i] || !comms[i]->nc || comms[i]->nranks != nranks) return set_error(err, RS16_INVALID_ARGUMENT);
    const bool virt = vslices > 0;
    if (virt && (nranks != 1 || n != 1 || vslices > 4096)) return set_error(err, RS16_INVALID_ARGUMENT);
    const int P = virt ? vslices : nranks;
    auto owner = [&](int j) { return virt ? 0 : j; };
    // the slice that the root keeps without RCCL: its own (slice 0 when virtual)
    const int own = virt ? 0 : root;
    // buffer of slice j on local communicator i (which owns it)
    auto slice_buf = [&](int i, int j) { return virt ? d_slice[j] : d_slice[i]; };
    auto strm = [&](rs16_comm* c) { return (n == 1 && stream) ? (hipStream_t)stream : c->eng->stream; };
    // root: its own slice directly; scatter: pack every other slice (one
    // pitched copy each)
    for (int i = 0; i < n; i++) {
        rs16_comm* c = comms[i];
        if (c->rank != root) continue;
        if (int rc = c->eng->activate(err)) return rc;
        size_t off, w;
        col_slice(S, P, own, &off, &w);
        if (w && scatter)
            RS16_HIP(hipMemcpy2DAsync(slice_buf(i, own), w, (const uint8_t*)d_full[i] + off, S, w, rows,
                                      hipMemcpyDeviceToDevice, strm(c)));
        if (w && !scatter)
            RS16_HIP(hipMemcpy2DAsync((uint8_t*)d_full[i] + off, S, slice_buf(i, own), w, w, rows,
                                      hipMemcpyDeviceToDevice, strm(c)));
        if (P == 1) continue;
        // the previous collective's use of the staging buffer (maybe on another stream)
        if (c->stage_busy) RS16_HIP(hipStreamWaitEvent(strm(c), c->stage_ev, 0));
        if (c->stage.cap < rows * S) {
            RS16_HIP(hipStreamSynchronize(strm(c)));  // (reserve frees the old buffer)
            RS16_HIP(c->stage.reserve(rows * S));
        }
        if (scatter)
            for (int j = 0; j < P; j++) {
                col_slice(S, P, j, &off, &w);
                if (!w || j == own) continue;
                RS16_HIP(hipMemcpy2DAsync((uint8_t*)c->stage.p + rows * off, w, (const uint8_t*)d_full[i] + off, S, w,
                                          rows, hipMemcpyDeviceToDevice, strm(c)));
            }
    }
    if (P == 1) return set_error(err, RS16_OK);
    RS16_NCCL(ncclGroupStart());
    auto p2p = [&](bool send, void* p, size_t bytes, int peer, rs16_comm* c) -> int {
        const ncclResult_t x = send ? ncclSend(p, bytes, ncclUint8, peer, c->nc, strm(c))
                                    : ncclRecv(p, bytes, ncclUint8, peer, c->nc, strm(c));
        if (x != ncclSuccess) {
            (void)ncclGroupEnd();
            return nccl_fail(err, x);
        }
        return RS16_OK;
    };
    for (int i = 0; i < n; i++) {
        rs16_comm* c = comms[i];
        if (int rc = c->eng->activate(err)) {
            (void)ncclGroupEnd();
            return rc;
        }
        // the root's side: one send (scatter) / receive (gather) per slice it does not keep
        if (c->rank == root)
            for (int j = 0; j < P; j++) {
                size_t o2, w2;
                col_slice(S, P, j, &o2, &w2);
                if (!w2 || j == own) continue;
                if (int rc = p2p(scatter, (uint8_t*)c->stage.p + rows * o2, rows * w2, owner(j), c)) return rc;
            }
        // the owners' side: every slice of this rank that the root does not keep
        for (int j = 0; j < P; j++) {
            if (owner(j) != c->rank || j == own) continue;
            size_t o2, w2;
            col_slice(S, P, j, &o2, &w2);
            if (!w2) continue;
            if (int rc = p2p(!scatter, slice_buf(i, j), rows * w2, root, c)) return rc;
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
    // root, gather: unpack into the full rows x S array; then mark the
    // staging buffer's last use (both directions)
    for (int i = 0; i < n; i++) {
        rs16_comm* c = comms[i];
        if (c->rank != root) continue;
        if (int rc = c->eng->activate(err)) return rc;
        if (!scatter)
            for (int j = 0; j < P; j++) {
                size_t off, w;
                col_slice(S, P, j, &off, &w);
                if (!w || j == own) continue;
                RS16_HIP(hipMemcpy2DAsync((uint8_t*)d_full[i] + off, S, (const uint8_t*)c->stage.p + rows * off, w, w,
                                          rows, hipMemcpyDeviceToDevice, strm(c)));
            }
        if (!c->stage_ev) RS16_HIP(hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming));
        RS16_HIP(hipEventRecord(c->stage_ev, strm(c)));
        c->stage_busy = true;
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

// Diagnostics (include/rs16.h): the multi-rank data path with `vslices`
// virtual slices, all owned by the one rank of `comm`.
extern "C" int rs16_scatter_columns_virtual(rs16_comm* comm, int vslices, size_t rows, size_t shard_bytes,
                                            const void* d_full, void* const* d_slices, void* stream,
                                            rs16_error* err) {
    if (!comm || vslices < 1 || !d_slices) return set_error(err, RS16_INVALID_ARGUMENT);
    void* full = (void*)d_full;
    return columns(&comm, 1, 0, rows, shard_bytes, &full, d_slices, stream, true, err, vslices);
}
extern "C" int rs16_gather_columns_virtual(rs16_comm* comm, int vslices, size_t rows, size_t shard_bytes,
                                           const void* const* d_slices, void* d_full, void* stream, rs16_error* err) {
    if (!comm || vslices < 1 || !d_slices) return set_error(err, RS16_INVALID_ARGUMENT);
    return columns(&comm, 1, 0, rows, shard_bytes, &d_full, (void* const*)d_slices, stream, false, err, vslices);
}
