/*
 * oracle/sigoracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C restatement of syzkaller's coverage-signal path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg to check and time the
 * MI355X product (libsyzsig.so).  Nothing in syzkaller_amd/ links or loads this.
 *
 * Every function names the reference lines it follows (paths relative to the
 * reference checkout).  The reference is Go (pkg/cover, syz-fuzzer, syz-manager)
 * plus C++ (executor); no Go toolchain exists in this image, so the Go parts are
 * restated here and pinned by the known-answer tests in pkg/cover/cover_test.go
 * (tests/golden/cover_kats.json).  The executor part is additionally pinned by
 * the compiled reference executor (oracle/_ref, see oracle/Makefile).
 *
 * Go `map[uint32]struct{}` is mirrored by an open-addressing hash set (orc_set)
 * so that the CPU baseline pays the same kind of per-element probe cost as the
 * reference does.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SENT 0xFFFFFFFFu /* pkg/cover/cover.go:17  const sent = ^uint32(0) */

/* ------------------------------------------------------------------------- */
/* pkg/cover/cover.go:28-40  Canonicalize: sort.Sort ascending, then unique;  */
/* `last` starts at sent so 0xFFFFFFFF is dropped.  In place, returns new n.  */
/* (sort order of equal uint32 values is unobservable, so any sort is exact.) */
/* ------------------------------------------------------------------------- */
static void radix_sort_u32(uint32_t* v, size_t n)
{
	if (n < 64) { /* insertion sort for tiny inputs */
		for (size_t i = 1; i < n; i++) {
			uint32_t x = v[i];
			size_t j = i;
			while (j > 0 && v[j - 1] > x) {
				v[j] = v[j - 1];
				j--;
			}
			v[j] = x;
		}
		return;
	}
	uint32_t* tmp = (uint32_t*)malloc(n * sizeof(uint32_t));
	uint32_t* src = v;
	uint32_t* dst = tmp;
	for (int shift = 0; shift < 32; shift += 8) {
		size_t cnt[256] = {0};
		for (size_t i = 0; i < n; i++)
			cnt[(src[i] >> shift) & 0xFF]++;
		size_t sum = 0;
		for (int b = 0; b < 256; b++) {
			size_t c = cnt[b];
			cnt[b] = sum;
			sum += c;
		}
		for (size_t i = 0; i < n; i++)
			dst[cnt[(src[i] >> shift) & 0xFF]++] = src[i];
		uint32_t* t = src;
		src = dst;
		dst = t;
	}
	/* four passes: result is back in v */
	free(tmp);
}

size_t orc_canonicalize(uint32_t* v, size_t n)
{
	radix_sort_u32(v, n);
	size_t i = 0;
	uint32_t last = SENT;
	for (size_t k = 0; k < n; k++) {
		if (v[k] != last) {
			last = v[k];
			v[i++] = v[k];
		}
	}
	return i;
}

/* ------------------------------------------------------------------------- */
/* pkg/cover/cover.go:42-102  Difference / SymmetricDifference / Union /      */
/* Intersection, all through foreach (cover.go:81-102).  out capacity na+nb.  */
/* ------------------------------------------------------------------------- */
enum { ORC_DIFF = 0, ORC_SYMDIFF = 1, ORC_UNION = 2, ORC_INTER = 3 };

static inline uint32_t orc_apply(int op, uint32_t v0, uint32_t v1)
{
	switch (op) {
	case ORC_DIFF: /* cover.go:43-48 */
		return v0 < v1 ? v0 : SENT;
	case ORC_SYMDIFF: /* cover.go:52-60 */
		if (v0 < v1)
			return v0;
		if (v1 < v0)
			return v1;
		return SENT;
	case ORC_UNION: /* cover.go:64-69 */
		return v0 <= v1 ? v0 : v1;
	default: /* ORC_INTER, cover.go:73-78 */
		return v0 == v1 ? v0 : SENT;
	}
}

size_t orc_foreach(int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out)
{
	size_t n = 0;
	size_t i0 = 0, i1 = 0;
	while (i0 < na || i1 < nb) { /* cover.go:83 */
		uint32_t v0 = SENT, v1 = SENT;
		if (i0 < na)
			v0 = a[i0];
		if (i1 < nb)
			v1 = b[i1];
		if (v0 <= v1)
			i0++;
		if (v1 <= v0)
			i1++;
		uint32_t v = orc_apply(op, v0, v1);
		if (v != SENT) /* cover.go:97 */
			out[n++] = v;
	}
	return n;
}

/* pkg/cover/cover.go:106-117  HasDifference (no sentinel special case). */
int orc_has_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb)
{
	size_t i1 = 0;
	for (size_t i0 = 0; i0 < na; i0++) {
		uint32_t v0 = a[i0];
		while (i1 < nb && b[i1] < v0)
			i1++;
		if (i1 == nb || b[i1] > v0)
			return 1;
		i1++;
	}
	return 0;
}

/* ------------------------------------------------------------------------- */
/* Go map[uint32]struct{} mirror: open addressing, linear probing.            */
/* ------------------------------------------------------------------------- */
typedef struct orc_set {
	uint64_t* slot; /* EMPTY or the key */
	size_t cap;     /* power of two */
	size_t count;
} orc_set;

#define ORC_EMPTY 0xFFFFFFFFFFFFFFFFull

static inline size_t orc_h(uint32_t k, size_t mask)
{
	uint64_t x = (uint64_t)k * 0x9E3779B97F4A7C15ull;
	return (size_t)(x >> 32) & mask;
}

orc_set* orc_set_new(void)
{
	orc_set* s = (orc_set*)calloc(1, sizeof(orc_set));
	s->cap = 1024;
	s->slot = (uint64_t*)malloc(s->cap * sizeof(uint64_t));
	memset(s->slot, 0xFF, s->cap * sizeof(uint64_t));
	return s;
}

void orc_set_free(orc_set* s)
{
	if (!s)
		return;
	free(s->slot);
	free(s);
}

size_t orc_set_count(const orc_set* s) { return s->count; }

int orc_set_has(const orc_set* s, uint32_t k)
{
	size_t mask = s->cap - 1;
	for (size_t p = orc_h(k, mask);; p = (p + 1) & mask) {
		uint64_t v = s->slot[p];
		if (v == ORC_EMPTY)
			return 0;
		if (v == k)
			return 1;
	}
}

static void orc_set_grow(orc_set* s)
{
	size_t ocap = s->cap;
	uint64_t* old = s->slot;
	s->cap = ocap * 2;
	s->slot = (uint64_t*)malloc(s->cap * sizeof(uint64_t));
	memset(s->slot, 0xFF, s->cap * sizeof(uint64_t));
	size_t mask = s->cap - 1;
	for (size_t i = 0; i < ocap; i++) {
		if (old[i] == ORC_EMPTY)
			continue;
		size_t p = orc_h((uint32_t)old[i], mask);
		while (s->slot[p] != ORC_EMPTY)
			p = (p + 1) & mask;
		s->slot[p] = old[i];
	}
	free(old);
}

void orc_set_add1(orc_set* s, uint32_t k)
{
	if ((s->count + 1) * 2 > s->cap)
		orc_set_grow(s);
	size_t mask = s->cap - 1;
	for (size_t p = orc_h(k, mask);; p = (p + 1) & mask) {
		uint64_t v = s->slot[p];
		if (v == k)
			return;
		if (v == ORC_EMPTY) {
			s->slot[p] = k;
			s->count++;
			return;
		}
	}
}

/* Export all keys in ascending order (the product's export order). */
size_t orc_set_export(const orc_set* s, uint32_t* out)
{
	size_t n = 0;
	for (size_t i = 0; i < s->cap; i++)
		if (s->slot[i] != ORC_EMPTY)
			out[n++] = (uint32_t)s->slot[i];
	radix_sort_u32(out, n);
	return n;
}

/* pkg/cover/cover.go:160-167  SignalNew */
int orc_signal_new(const orc_set* base, const uint32_t* sig, size_t n)
{
	for (size_t i = 0; i < n; i++)
		if (!orc_set_has(base, sig[i]))
			return 1;
	return 0;
}

/* pkg/cover/cover.go:169-176  SignalDiff (order and duplicates kept) */
size_t orc_signal_diff(const orc_set* base, const uint32_t* sig, size_t n, uint32_t* out)
{
	size_t m = 0;
	for (size_t i = 0; i < n; i++)
		if (!orc_set_has(base, sig[i]))
			out[m++] = sig[i];
	return m;
}

/* pkg/cover/cover.go:178-182  SignalAdd */
void orc_signal_add(orc_set* base, const uint32_t* sig, size_t n)
{
	for (size_t i = 0; i < n; i++)
		orc_set_add1(base, sig[i]);
}

/* ------------------------------------------------------------------------- */
/* syz-fuzzer/fuzzer.go:645-693  execute(): the per-call new-signal check,    */
/* run over a batch of call records in sequential (program-major, call-index) */
/* order.  rec_new[r] = 1 iff record r would be queued for triage             */
/* (fuzzer.go:678-690); its diff (fuzzer.go:669) is written to diff_vals at   */
/* diff_off[r] when those are non-NULL.  maxset/newset are updated exactly as */
/* fuzzer.go:673-674.                                                          */
/* ------------------------------------------------------------------------- */
uint64_t orc_triage_batch(orc_set* maxset, orc_set* newset, const uint32_t* vals, const uint64_t* rec_off,
			  size_t nrec, uint8_t* rec_new, uint32_t* diff_vals, uint64_t* diff_off)
{
	uint64_t nd = 0;
	uint32_t* tmp = NULL;
	size_t tmpcap = 0;
	for (size_t r = 0; r < nrec; r++) {
		const uint32_t* sig = vals + rec_off[r];
		size_t n = (size_t)(rec_off[r + 1] - rec_off[r]);
		if (diff_off)
			diff_off[r] = nd;
		rec_new[r] = 0;
		if (!orc_signal_new(maxset, sig, n)) /* fuzzer.go:666 */
			continue;
		uint32_t* d;
		if (diff_vals) {
			d = diff_vals + nd;
		} else {
			if (tmpcap < n) {
				free(tmp);
				tmpcap = n;
				tmp = (uint32_t*)malloc(tmpcap * sizeof(uint32_t));
			}
			d = tmp;
		}
		size_t m = orc_signal_diff(maxset, sig, n, d); /* fuzzer.go:669 */
		orc_signal_add(maxset, d, m);                   /* fuzzer.go:673 */
		if (newset)
			orc_signal_add(newset, d, m); /* fuzzer.go:674 */
		rec_new[r] = 1;
		nd += m;
	}
	if (diff_off)
		diff_off[nrec] = nd;
	free(tmp);
	return nd;
}

/* ------------------------------------------------------------------------- */
/* The fuzzer's concurrent form, for the CPU baseline's all-cores leg only:   */
/* nthreads "procs" (syz-fuzzer/fuzzer.go:248-327) each take whole programs   */
/* from a shared counter and run execute()'s loop (fuzzer.go:661-691) over    */
/* their calls, sharing maxSignal / newSignal under one reader-writer lock    */
/* (signalMu, fuzzer.go:65): RLock for SignalNew / SignalDiff, the RUnlock -> */
/* Lock upgrade for the two SignalAdd (fuzzer.go:671-676).  As in the         */
/* reference, the outcome depends on the interleaving (two procs can triage   */
/* the same signal in the upgrade window); it is timed, never compared.       */
/* ------------------------------------------------------------------------- */
typedef struct {
	orc_set *maxset, *newset;
	const uint32_t* vals;
	const uint64_t* rec_off;
	const uint64_t* prog_rec; /* program p owns records prog_rec[p] .. prog_rec[p+1] */
	size_t nprog;
	uint8_t* rec_new;
	pthread_rwlock_t mu;
	size_t next; /* next program, taken under __atomic */
} orc_procs;

static void* orc_proc_main(void* arg)
{
	orc_procs* a = (orc_procs*)arg;
	uint32_t* diff = NULL;
	size_t cap = 0;
	for (;;) {
		size_t p = __atomic_fetch_add(&a->next, 1, __ATOMIC_RELAXED);
		if (p >= a->nprog)
			break;
		pthread_rwlock_rdlock(&a->mu); /* fuzzer.go:662 */
		for (uint64_t r = a->prog_rec[p]; r < a->prog_rec[p + 1]; r++) {
			const uint32_t* sig = a->vals + a->rec_off[r];
			size_t n = (size_t)(a->rec_off[r + 1] - a->rec_off[r]);
			a->rec_new[r] = 0;
			if (!orc_signal_new(a->maxset, sig, n)) /* fuzzer.go:666 */
				continue;
			if (cap < n) {
				free(diff);
				cap = n;
				diff = (uint32_t*)malloc(cap * sizeof(uint32_t));
			}
			size_t m = orc_signal_diff(a->maxset, sig, n, diff); /* fuzzer.go:669 */
			pthread_rwlock_unlock(&a->mu);                       /* fuzzer.go:671-672 */
			pthread_rwlock_wrlock(&a->mu);
			orc_signal_add(a->maxset, diff, m); /* fuzzer.go:673-674 */
			if (a->newset)
				orc_signal_add(a->newset, diff, m);
			pthread_rwlock_unlock(&a->mu); /* fuzzer.go:675-676 */
			pthread_rwlock_rdlock(&a->mu);
			a->rec_new[r] = 1;
		}
		pthread_rwlock_unlock(&a->mu);
	}
	free(diff);
	return NULL;
}

/* Returns the number of threads that ran. */
int orc_triage_procs(orc_set* maxset, orc_set* newset, const uint32_t* vals, const uint64_t* rec_off,
		     const uint64_t* prog_rec, size_t nprog, int nthreads, uint8_t* rec_new)
{
	orc_procs a;
	memset(&a, 0, sizeof(a));
	a.maxset = maxset;
	a.newset = newset;
	a.vals = vals;
	a.rec_off = rec_off;
	a.prog_rec = prog_rec;
	a.nprog = nprog;
	a.rec_new = rec_new;
	pthread_rwlock_init(&a.mu, NULL);
	if (nthreads < 1)
		nthreads = 1;
	pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
	int started = 0;
	for (int i = 0; i < nthreads; i++)
		if (pthread_create(&th[i], NULL, orc_proc_main, &a) == 0)
			started++;
		else
			break;
	if (started == 0)
		orc_proc_main(&a);
	for (int i = 0; i < started; i++)
		pthread_join(th[i], NULL);
	free(th);
	pthread_rwlock_destroy(&a.mu);
	return started ? started : 1;
}

/* syz-fuzzer/fuzzer.go:467-489  addInput(): per input, in order. */
void orc_add_inputs(orc_set* corpus, orc_set* maxset, const uint32_t* vals, const uint64_t* off, size_t n)
{
	uint32_t* tmp = NULL;
	size_t tmpcap = 0;
	for (size_t k = 0; k < n; k++) {
		const uint32_t* sig = vals + off[k];
		size_t len = (size_t)(off[k + 1] - off[k]);
		if (tmpcap < len) {
			free(tmp);
			tmpcap = len;
			tmp = (uint32_t*)malloc(tmpcap * sizeof(uint32_t));
		}
		size_t m = orc_signal_diff(maxset, sig, len, tmp); /* fuzzer.go:485 */
		if (m) {
			orc_signal_add(corpus, tmp, m); /* fuzzer.go:486 */
			orc_signal_add(maxset, tmp, m); /* fuzzer.go:487 */
		}
	}
	free(tmp);
}

/* syz-manager/manager.go:907-912  NewInput acceptance, over a batch of RPCs */
/* in arrival order.  cov_* may be NULL (no cover tracked).                   */
void orc_accept_batch(orc_set* corpus_sig, orc_set* corpus_cov, const uint32_t* sig_vals, const uint64_t* sig_off,
		      const uint32_t* cov_vals, const uint64_t* cov_off, size_t n, uint8_t* accepted)
{
	for (size_t k = 0; k < n; k++) {
		const uint32_t* s = sig_vals + sig_off[k];
		size_t len = (size_t)(sig_off[k + 1] - sig_off[k]);
		accepted[k] = 0;
		if (!orc_signal_new(corpus_sig, s, len)) /* manager.go:907 */
			continue;
		accepted[k] = 1;
		orc_signal_add(corpus_sig, s, len); /* manager.go:911 */
		if (corpus_cov && cov_vals)
			orc_signal_add(corpus_cov, cov_vals + cov_off[k],
				       (size_t)(cov_off[k + 1] - cov_off[k])); /* manager.go:912 */
	}
}

/* syz-manager/manager.go:949-956  Poll maxSignal merge, batched over polls in */
/* arrival order (CSR a_vals/a_off).  new_vals gets the newMaxSignal lists,    */
/* new_off their offsets.  Returns the total.                                  */
uint64_t orc_merge_poll(orc_set* mgr_max, const uint32_t* a_vals, const uint64_t* a_off, size_t npoll,
			uint32_t* new_vals, uint64_t* new_off)
{
	uint64_t m = 0;
	for (size_t k = 0; k < npoll; k++) {
		new_off[k] = m;
		for (uint64_t i = a_off[k]; i < a_off[k + 1]; i++) {
			uint32_t s = a_vals[i];
			if (orc_set_has(mgr_max, s)) /* manager.go:950-952 */
				continue;
			orc_set_add1(mgr_max, s); /* manager.go:953 */
			new_vals[m++] = s;        /* manager.go:954 */
		}
	}
	new_off[npoll] = m;
	return m;
}

/* ------------------------------------------------------------------------- */
/* Go 1.8/1.9 sort.Sort (quickSort + ShellSort-gap-6 + insertionSort +        */
/* heapSort), restated from the published algorithm of the Go standard       */
/* library `sort` package (sort.go); used for minInputArray ordering          */
/* (pkg/cover/cover.go:128, Less at cover.go:157: len(a[i]) > len(a[j])).     */
/* Operates on an index permutation `p` with key `len`.                       */
/* ------------------------------------------------------------------------- */
typedef struct {
	uint32_t* p;
	const uint64_t* len;
} gosort_t;

static inline int gs_less(gosort_t* d, long i, long j) { return d->len[d->p[i]] > d->len[d->p[j]]; }
static inline void gs_swap(gosort_t* d, long i, long j)
{
	uint32_t t = d->p[i];
	d->p[i] = d->p[j];
	d->p[j] = t;
}

static void gs_insertion(gosort_t* d, long a, long b)
{
	for (long i = a + 1; i < b; i++)
		for (long j = i; j > a && gs_less(d, j, j - 1); j--)
			gs_swap(d, j, j - 1);
}

static void gs_sift_down(gosort_t* d, long lo, long hi, long first)
{
	long root = lo;
	for (;;) {
		long child = 2 * root + 1;
		if (child >= hi)
			break;
		if (child + 1 < hi && gs_less(d, first + child, first + child + 1))
			child++;
		if (!gs_less(d, first + root, first + child))
			return;
		gs_swap(d, first + root, first + child);
		root = child;
	}
}

static void gs_heap(gosort_t* d, long a, long b)
{
	long first = a, lo = 0, hi = b - a;
	for (long i = (hi - 1) / 2; i >= 0; i--)
		gs_sift_down(d, i, hi, first);
	for (long i = hi - 1; i >= 0; i--) {
		gs_swap(d, first, first + i);
		gs_sift_down(d, lo, i, first);
	}
}

static void gs_median3(gosort_t* d, long m1, long m0, long m2)
{
	if (gs_less(d, m1, m0))
		gs_swap(d, m1, m0);
	if (gs_less(d, m2, m1)) {
		gs_swap(d, m2, m1);
		if (gs_less(d, m1, m0))
			gs_swap(d, m1, m0);
	}
}

static void gs_pivot(gosort_t* d, long lo, long hi, long* midlo, long* midhi)
{
	long m = (long)(((unsigned long)(lo + hi)) >> 1);
	if (hi - lo > 40) {
		long s = (hi - lo) / 8;
		gs_median3(d, lo, lo + s, lo + 2 * s);
		gs_median3(d, m, m - s, m + s);
		gs_median3(d, hi - 1, hi - 1 - s, hi - 1 - 2 * s);
	}
	gs_median3(d, lo, m, hi - 1);
	long pivot = lo;
	long a = lo + 1, c = hi - 1;
	for (; a < c && gs_less(d, a, pivot); a++) {
	}
	long b = a;
	for (;;) {
		for (; b < c && !gs_less(d, pivot, b); b++) {
		}
		for (; b < c && gs_less(d, pivot, c - 1); c--) {
		}
		if (b >= c)
			break;
		gs_swap(d, b, c - 1);
		b++;
		c--;
	}
	int protect = hi - c < 5;
	if (!protect && hi - c < (hi - lo) / 4) {
		int dups = 0;
		if (!gs_less(d, pivot, hi - 1)) {
			gs_swap(d, c, hi - 1);
			c++;
			dups++;
		}
		if (!gs_less(d, b - 1, pivot)) {
			b--;
			dups++;
		}
		if (!gs_less(d, m, pivot)) {
			gs_swap(d, m, b - 1);
			b--;
			dups++;
		}
		protect = dups > 1;
	}
	if (protect) {
		for (;;) {
			for (; a < b && !gs_less(d, b - 1, pivot); b--) {
			}
			for (; a < b && gs_less(d, a, pivot); a++) {
			}
			if (a >= b)
				break;
			gs_swap(d, a, b - 1);
			a++;
			b--;
		}
	}
	gs_swap(d, pivot, b - 1);
	*midlo = b - 1;
	*midhi = c;
}

static void gs_quick(gosort_t* d, long a, long b, int maxdepth)
{
	while (b - a > 12) {
		if (maxdepth == 0) {
			gs_heap(d, a, b);
			return;
		}
		maxdepth--;
		long mlo, mhi;
		gs_pivot(d, a, b, &mlo, &mhi);
		if (mlo - a < b - mhi) {
			gs_quick(d, a, mlo, maxdepth);
			a = mhi;
		} else {
			gs_quick(d, mhi, b, maxdepth);
			b = mlo;
		}
	}
	if (b - a > 1) {
		for (long i = a + 6; i < b; i++)
			if (gs_less(d, i, i - 6))
				gs_swap(d, i, i - 6);
		gs_insertion(d, a, b);
	}
}

/* order[k] = index of the input processed k-th by cover.Minimize. */
void orc_minimize_order(const uint64_t* off, size_t n, uint32_t* order)
{
	uint64_t* len = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
	for (size_t i = 0; i < n; i++) {
		len[i] = off[i + 1] - off[i];
		order[i] = (uint32_t)i;
	}
	gosort_t d = {order, len};
	int depth = 0;
	for (size_t i = n; i > 0; i >>= 1)
		depth++;
	gs_quick(&d, 0, (long)n, depth * 2);
	free(len);
}

/* pkg/cover/cover.go:129-145  Minimize's greedy loop over a given order.     */
/* Returns the number of selected inputs; out_idx gets them in rank order.    */
size_t orc_minimize_ordered(const uint32_t* vals, const uint64_t* off, size_t n, const uint32_t* order,
			    uint32_t* out_idx)
{
	orc_set* covered = orc_set_new();
	size_t nmin = 0;
	for (size_t k = 0; k < n; k++) {
		uint32_t idx = order[k];
		int hit = 0;
		for (uint64_t i = off[idx]; i < off[idx + 1]; i++) {
			uint32_t pc = vals[i];
			if (!hit && !orc_set_has(covered, pc)) { /* cover.go:134-138 */
				hit = 1;
				out_idx[nmin++] = idx;
			}
			if (hit)
				orc_set_add1(covered, pc); /* cover.go:140-142 */
		}
	}
	orc_set_free(covered);
	return nmin;
}

/* ------------------------------------------------------------------------- */
/* executor/executor.h:497-526  hash() and dedup(); executor.h:389-401 the    */
/* per-call edge-signal loop.  One dedup table per program (the executor      */
/* forks a child per program, executor/executor_linux.cc:174), shared by all  */
/* of that program's calls, handled in call order.                            */
/* ------------------------------------------------------------------------- */
#define ORC_DEDUP_SIZE 8192u

uint32_t orc_exec_hash(uint32_t a)
{
	a = (a ^ 61) ^ (a >> 16);
	a = a + (a << 3);
	a = a ^ (a >> 4);
	a = a * 0x27d4eb2du;
	a = a ^ (a >> 15);
	return a;
}

static int orc_exec_dedup(uint32_t* table, uint32_t sig)
{
	for (uint32_t i = 0; i < 4; i++) {
		uint32_t pos = (sig + i) % ORC_DEDUP_SIZE;
		if (table[pos] == sig)
			return 1;
		if (table[pos] == 0) {
			table[pos] = sig;
			return 0;
		}
	}
	table[sig % ORC_DEDUP_SIZE] = sig;
	return 0;
}

/* Batch: programs p own calls [prog_off[p], prog_off[p+1]); call c owns PCs  */
/* [call_off[c], call_off[c+1]).  Emitted signal of call c goes to            */
/* out[sig_off[c] .. sig_off[c+1]); out capacity = total PCs.  Returns total. */
uint64_t orc_exec_signal_batch(const uint32_t* pcs, const uint64_t* call_off, const uint64_t* prog_off, size_t nprog,
			       uint32_t* out, uint64_t* sig_off)
{
	uint32_t table[ORC_DEDUP_SIZE];
	uint64_t m = 0;
	for (size_t p = 0; p < nprog; p++) {
		memset(table, 0, sizeof(table));
		for (uint64_t c = prog_off[p]; c < prog_off[p + 1]; c++) {
			sig_off[c] = m;
			uint32_t prev = 0;
			for (uint64_t i = call_off[c]; i < call_off[c + 1]; i++) {
				uint32_t pc = pcs[i];
				uint32_t sig = pc ^ prev;
				prev = orc_exec_hash(pc);
				if (orc_exec_dedup(table, sig))
					continue;
				out[m++] = sig;
			}
		}
	}
	if (nprog)
		sig_off[prog_off[nprog]] = m;
	return m;
}

/* ------------------------------------------------------------------------- */
/* syz-manager/cover.go:91-103 + :257-307  cover report: pcs[i] =             */
/* RestorePC(cov[i], base) - callLen (pkg/cover/cover.go:23-25, callLen = 5   */
/* at syz-manager/cover.go:61), then uncoveredPcsInFuncs.  sym_start/sym_end  */
/* are sorted by start (syz-manager/cover.go:268).  The reference returns map */
/* order; the oracle returns the set ascending.  Returns the count.           */
/* ------------------------------------------------------------------------- */
static size_t lower_bound_u64(const uint64_t* a, size_t n, uint64_t key) /* first i: a[i] >= key */
{
	size_t lo = 0, hi = n;
	while (lo < hi) {
		size_t mid = lo + (hi - lo) / 2;
		if (a[mid] < key)
			lo = mid + 1;
		else
			hi = mid;
	}
	return lo;
}

static size_t upper_bound_u64(const uint64_t* a, size_t n, uint64_t key) /* first i: a[i] > key */
{
	size_t lo = 0, hi = n;
	while (lo < hi) {
		size_t mid = lo + (hi - lo) / 2;
		if (a[mid] <= key)
			lo = mid + 1;
		else
			hi = mid;
	}
	return lo;
}

size_t orc_cover_uncovered(const uint32_t* cov, size_t ncov, uint32_t base, const uint64_t* sym_start,
			   const uint64_t* sym_end, size_t nsym, const uint64_t* all_pcs, size_t nall, uint64_t* out)
{
	/* uncovered map and handledFuncs map mirrored by flag arrays. */
	uint8_t* unc = (uint8_t*)calloc(nall ? nall : 1, 1);
	uint8_t* handled = (uint8_t*)calloc(nsym ? nsym : 1, 1);
	/* map keys that are not in all_pcs can never be inserted, only deleted. */
	for (size_t k = 0; k < ncov; k++) {
		uint64_t pc = ((uint64_t)base << 32) + (uint64_t)cov[k] - 5; /* cover.go:101 */
		size_t idx = upper_bound_u64(sym_end, nsym, pc); /* sort.Search(pc < end), cover.go:278 */
		if (idx == nsym)
			continue;
		if (pc < sym_start[idx] || pc > sym_end[idx]) /* cover.go:285 */
			continue;
		/* handledFuncs is keyed by the symbol start (cover.go:288) */
		size_t key = lower_bound_u64(sym_start, nsym, sym_start[idx]);
		if (!handled[key]) { /* cover.go:288-298 */
			handled[key] = 1;
			size_t lo = lower_bound_u64(all_pcs, nall, sym_start[idx]);
			size_t hi = upper_bound_u64(all_pcs, nall, sym_end[idx]);
			for (size_t j = lo; j < hi; j++)
				unc[j] = 1;
		}
		/* delete(uncovered, pc), cover.go:299 */
		size_t j = lower_bound_u64(all_pcs, nall, pc);
		while (j < nall && all_pcs[j] == pc) {
			unc[j] = 0;
			j++;
		}
	}
	size_t n = 0;
	for (size_t j = 0; j < nall; j++)
		if (unc[j] && (n == 0 || out[n - 1] != all_pcs[j]))
			out[n++] = all_pcs[j];
	free(unc);
	free(handled);
	return n;
}
