/* oracle/aq_bag.c -- TEST INFRASTRUCTURE ONLY (CPU baseline / checker; never linked into the product).
 *
 * The reference's bag of tasks restated with threads instead of MPI ranks: the
 * same-host CPU baseline when the reference binary (oracle/_ref, built from /root/reference) cannot
 * run. One farmer thread and P-1 worker threads, P = "-n" like mpirun -n:
 *   farmer  /root/reference/aquadPartA.c:125-173  LIFO bag seeded with [A,B] (:134-137); every
 *           message from a worker marks it idle (:146-147); an accepted area is added in arrival
 *           order (:148-149), a refining task's two children are pushed in send order (:151-154);
 *           then idle workers are scanned round-robin from worker 0 and each gets pop(bag)
 *           (:157-165), counting tasks_per_process[j+1] (:162); done when the bag is empty and every
 *           worker is idle (:166), then every worker is told to exit (:167-171).
 *   worker  :175-205  the task body verbatim: lrarea, mid, fmid, larea, rarea, strict '>' against
 *           EPSILON (:185-191); children [l,mid], [mid,r] (:192-197) or the area larea+rarea (:199).
 *   main    :107-117  the same stdout: "Area=%lf", blank line, "Tasks Per Process", the index row and
 *           the count row, tab-separated; P < 2 -> the reference's error message and exit 1 (:86-90).
 * F is the host libm's, exactly as the reference evaluates it (cosh^4 :46, or sin(1/x) for config 4).
 * MPI_Recv(ANY_SOURCE) becomes a scan of per-worker outboxes, MPI_Send a per-worker inbox; both are
 * single-producer single-consumer slots with release/acquire flags, and every thread busy-polls,
 * as MPICH's shared-memory channel does.
 *
 *   aq_bag [-n P] [-e EPSILON] [-a A] [-b B] [-f cosh4|sin]
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static double EPS = 1e-3, A = 0.0, B = 5.0;
static int SIN_RECIP = 0;

static double F(double x) {
    if (SIN_RECIP) return sin(1.0 / x);
    return cosh(x) * cosh(x) * cosh(x) * cosh(x);   /* :46, left to right */
}

typedef struct {
    _Alignas(64) atomic_int in_flag;   /* 1: task in l/r, 2: exit */
    double l, r;
    _Alignas(64) atomic_int out_flag;  /* 1: message in tag/buf */
    int tag;                           /* 1 area, 0 two children */
    double buf[4];
} mbox;

static mbox* boxes;

static void relax(unsigned* spins) {
    if (++*spins > 4096u) {
        sched_yield();
        *spins = 0;
    }
}

static void* worker(void* arg) {
    mbox* m = &boxes[(size_t)arg];
    unsigned spins = 0;
    /* the initial "I am idle" message (:178) */
    m->tag = 1;
    m->buf[0] = 0.0;
    atomic_store_explicit(&m->out_flag, 1, memory_order_release);
    for (;;) {
        int f;
        while ((f = atomic_load_explicit(&m->in_flag, memory_order_acquire)) == 0) relax(&spins);
        if (f == 2) break;
        const double left = m->l, right = m->r;
        atomic_store_explicit(&m->in_flag, 0, memory_order_relaxed);
        const double lrarea = (F(left) + F(right)) * (right - left) / 2;   /* :185 */
        const double mid = (left + right) / 2;                             /* :187 */
        const double fmid = F(mid);                                        /* :188 */
        const double larea = (F(left) + fmid) * (mid - left) / 2;          /* :189 */
        const double rarea = (fmid + F(right)) * (right - mid) / 2;        /* :190 */
        while (atomic_load_explicit(&m->out_flag, memory_order_acquire)) relax(&spins);
        if (fabs((larea + rarea) - lrarea) > EPS) {                       /* :191 */
            m->tag = 0;
            m->buf[0] = left; m->buf[1] = mid;                              /* :193-195 */
            m->buf[2] = mid;  m->buf[3] = right;                            /* :196-198 */
        } else {
            m->tag = 1;
            m->buf[0] = larea + rarea;                                      /* :199-201 */
        }
        atomic_store_explicit(&m->out_flag, 1, memory_order_release);
    }
    return NULL;
}

typedef struct { double* v; size_t n, cap; } stack;   /* the bag: (l, r) pairs, LIFO */

static void push(stack* s, double l, double r) {
    if (s->n == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 1024;
        s->v = (double*)realloc(s->v, 2 * s->cap * sizeof(double));
        if (!s->v) { perror("aq_bag"); exit(1); }
    }
    s->v[2 * s->n] = l;
    s->v[2 * s->n + 1] = r;
    s->n++;
}

int main(int argc, char** argv) {
    int nprocs = 5;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "-n")) nprocs = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-e")) EPS = atof(argv[i + 1]);
        else if (!strcmp(argv[i], "-a")) A = atof(argv[i + 1]);
        else if (!strcmp(argv[i], "-b")) B = atof(argv[i + 1]);
        else if (!strcmp(argv[i], "-f")) SIN_RECIP = !strcmp(argv[i + 1], "sin");
    }
    if (nprocs < 2) {   /* :86-90 */
        fprintf(stderr, "ERROR: Must have at least 2 processes to run\n");
        return 1;
    }
    const int workers = nprocs - 1;
    boxes = (mbox*)aligned_alloc(64, sizeof(mbox) * (size_t)workers);
    memset(boxes, 0, sizeof(mbox) * (size_t)workers);
    int* tasks_per_process = (int*)calloc((size_t)nprocs, sizeof(int));
    int* idle = (int*)calloc((size_t)workers, sizeof(int));
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)workers);
    for (int w = 0; w < workers; ++w) pthread_create(&th[w], NULL, worker, (void*)(size_t)w);

    stack bag = {0};
    push(&bag, A, B);
    double result = 0.0;
    int idle_count = 0, scan = 0;
    unsigned spins = 0;
    do {
        /* MPI_Recv(ANY_SOURCE): the next outbox holding a message, scanning on from the last */
        int src = -1;
        while (src < 0) {
            for (int k = 0; k < workers; ++k) {
                const int w = (scan + k) % workers;
                if (atomic_load_explicit(&boxes[w].out_flag, memory_order_acquire)) { src = w; break; }
            }
            if (src < 0) relax(&spins);
        }
        scan = (src + 1) % workers;
        mbox* m = &boxes[src];
        idle_count++;                                   /* :146 */
        idle[src] = 1;                                  /* :147 */
        if (m->tag == 1) {
            result += m->buf[0];                        /* :149 */
        } else {
            push(&bag, m->buf[0], m->buf[1]);           /* :152 */
            push(&bag, m->buf[2], m->buf[3]);           /* :154 */
        }
        atomic_store_explicit(&m->out_flag, 0, memory_order_release);
        int j = 0;
        while (bag.n > 0 && idle_count > 0) {           /* :157 */
            if (idle[j]) {
                bag.n--;
                boxes[j].l = bag.v[2 * bag.n];
                boxes[j].r = bag.v[2 * bag.n + 1];
                atomic_store_explicit(&boxes[j].in_flag, 1, memory_order_release);
                idle[j] = 0;
                idle_count--;
                tasks_per_process[j + 1]++;             /* :162 */
            }
            j = (j + 1) % workers;
        }
    } while (bag.n > 0 || idle_count != workers);       /* :166 */
    for (int w = 0; w < workers; ++w) atomic_store_explicit(&boxes[w].in_flag, 2, memory_order_release);
    for (int w = 0; w < workers; ++w) pthread_join(th[w], NULL);

    fprintf(stdout, "Area=%lf\n", result);              /* :107-117 */
    fprintf(stdout, "\nTasks Per Process\n");
    for (int i = 0; i < nprocs; i++) fprintf(stdout, "%d\t", i);
    fprintf(stdout, "\n");
    for (int i = 0; i < nprocs; i++) fprintf(stdout, "%d\t", tasks_per_process[i]);
    fprintf(stdout, "\n");
    free(tasks_per_process);
    free(idle);
    free(th);
    free(bag.v);
    free(boxes);
    return 0;
}
