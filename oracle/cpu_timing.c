/*
 * oracle/cpu_timing.c — TEST / BENCH INFRASTRUCTURE ONLY.
 *
 * Times the oracle restatement of do_host_reduce<DT> (oracle_host_reduce, host_reduce.c; the reference
 * loop /root/reference/src/core/internal_common.hpp:496-586) on caller-owned host buffers, for bench.py's
 * CPU-baseline legs only (`cpu_baseline`, `host_crossover`).  The product path never links or calls it.
 *
 * The loop is timed in C so that a 4 KiB combine (a fraction of a microsecond) is not buried under a
 * Python call.  `nsets` operand pairs at `stride` bytes apart are combined in rotation, so a working set
 * larger than the last-level cache gives every call cold operands (as a chunk that just arrived by RDMA);
 * nsets == 1 repeats one pair (cache-resident when it fits).
 *
 * nthreads > 1 splits every combine into 64-B aligned contiguous slices over a persistent team (the
 * caller plus nthreads-1 pthreads) released and joined by a spinning generation barrier, the cheapest
 * dispatch a multi-threaded CPU combine could have; the reference itself runs one thread per rank.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <time.h>

int oracle_host_reduce(const void* send, void* recv, size_t count, int dtype, int op);

typedef struct {
    const unsigned char* send;
    unsigned char* recv;
    size_t stride, count, esz;
    int dtype, op, nthreads;
    size_t nsets;
    atomic_size_t set;      /* operand pair of the current round */
    atomic_uint gen;        /* bumped by the caller to start a round */
    atomic_uint done;       /* workers finished with the current round */
    atomic_int stop;
    atomic_int rc;
} Team;

typedef struct { Team* t; int id; } Arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void cpu_relax(void) { __builtin_ia32_pause(); }

/* thread `id`'s slice of the current pair: 64-B aligned contiguous, the last thread takes the remainder */
static void slice(Team* t, int id) {
    const size_t per_line = 64 / t->esz;
    const size_t per = t->count / (size_t)t->nthreads / per_line * per_line;
    const size_t b = per * (size_t)id, e = id == t->nthreads - 1 ? t->count : b + per;
    if (e <= b) return;
    const size_t s = atomic_load_explicit(&t->set, memory_order_relaxed) * t->stride;
    const int rc = oracle_host_reduce(t->send + s + b * t->esz, t->recv + s + b * t->esz, e - b, t->dtype, t->op);
    if (rc != 0) atomic_store(&t->rc, rc);
}

static void* worker(void* p) {
    Arg* a = (Arg*)p;
    Team* t = a->t;
    unsigned seen = 0;
    for (;;) {
        unsigned g;
        while ((g = atomic_load_explicit(&t->gen, memory_order_acquire)) == seen) cpu_relax();
        seen = g;
        if (atomic_load(&t->stop)) return NULL;
        slice(t, a->id);
        atomic_fetch_add_explicit(&t->done, 1, memory_order_acq_rel);
    }
}

/* One timed round over every thread: returns after all slices are combined. */
static void round_all(Team* t, size_t set) {
    atomic_store_explicit(&t->set, set, memory_order_relaxed);
    atomic_store_explicit(&t->done, 0, memory_order_relaxed);
    atomic_fetch_add_explicit(&t->gen, 1, memory_order_acq_rel);
    slice(t, 0);
    while (atomic_load_explicit(&t->done, memory_order_acquire) != (unsigned)(t->nthreads - 1)) cpu_relax();
}

/*
 * Seconds per combine of `count` elements, averaged over at least `min_seconds` and `min_reps` calls;
 * *reps_out receives the number of calls.  Returns a negative value on a bad argument or a failed
 * thread creation.
 */
double oracle_time_host_reduce(const void* send, void* recv, size_t nsets, size_t stride, size_t count, int dtype,
                               int op, int nthreads, double min_seconds, size_t min_reps, size_t* reps_out) {
    static const size_t esz_of[10] = {1, 1, 4, 4, 8, 8, 2, 4, 8, 2};
    if (dtype < 0 || dtype > 9 || nsets == 0 || nthreads < 1 || nthreads > 512 || count == 0) return -1.0;
    Team t;
    t.send = (const unsigned char*)send;
    t.recv = (unsigned char*)recv;
    t.stride = stride;
    t.count = count;
    t.esz = esz_of[dtype];
    t.dtype = dtype;
    t.op = op;
    t.nthreads = nthreads;
    t.nsets = nsets;
    atomic_init(&t.set, 0);
    atomic_init(&t.gen, 0);
    atomic_init(&t.done, 0);
    atomic_init(&t.stop, 0);
    atomic_init(&t.rc, 0);
    pthread_t th[512];
    Arg args[512];
    int started = 1;
    for (; started < nthreads; ++started) {
        args[started].t = &t;
        args[started].id = started;
        if (pthread_create(&th[started], NULL, worker, &args[started]) != 0) break;
    }
    double result = -1.0;
    size_t reps = 0;
    if (started == nthreads) {
        for (size_t i = 0; i < nsets && i < 4; ++i) round_all(&t, i);  /* warm the team and the first pairs */
        const double t0 = now_s();
        double el = 0.0;
        while (el < min_seconds || reps < min_reps) {
            round_all(&t, reps % nsets);
            ++reps;
            if ((reps & 15) == 0 || count >= (1u << 16)) el = now_s() - t0;
        }
        el = now_s() - t0;
        result = atomic_load(&t.rc) != 0 ? -2.0 : el / (double)reps;
    }
    atomic_store(&t.stop, 1);
    atomic_fetch_add_explicit(&t.gen, 1, memory_order_acq_rel);
    for (int i = 1; i < started; ++i) pthread_join(th[i], NULL);
    if (reps_out) *reps_out = reps;
    return result;
}
