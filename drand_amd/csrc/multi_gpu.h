// Multi-GPU batch verification behind the C ABI (dgpu_multi_open /
// dgpu_verify_multi).  Included at the end of capi.hip
// (one translation unit: the kernels and the context live there).
//
// The reference's bulk caller walks the chain serially
// (chain/beacon/sync_manager.go:188-222); every stored beacon carries its own
// PreviousSig (chain/beacon.go:15), so round verdicts are independent and the
// batch shards into contiguous round ranges, one per GPU, with no data-path
// collective.  RCCL over xGMI moves only results:
//  - per-round mode: one all-gather of the per-device verdict bitmaps (and
//    reason bytes) -- shards are multiples of 8 rounds, so the gathered
//    bitmaps concatenate into the batch's bitmap;
//  - RLC mode: one all-gather of the per-device RLC roots (two Jacobian sums
//    of the signature group: 672 bytes for G2 signatures, 336 for the G1
//    schemes; each computed by bucket MSM, rlc_msm.cuh), summed on
//    device 0 and checked there with a single pairing (one final
//    exponentiation for the whole node); only when that fails does each
//    device build its tree of leaves and descend it (root first) to
//    per-round verdicts, and the bitmaps are gathered as in per-round mode.
// RCCL is loaded at dgpu_multi_open (dlopen), so the single-GPU library has
// no link-time dependency on it.
//
// Test mode: with DGPU_MULTI_ALLOW_SAME_DEVICE=1 in the environment a handle
// may list one device several times (devs = {0, 0, 0}: one context each, own
// streams and buffers) and its all-gathers are in-library device copies
// ordered by events instead of RCCL (a communicator cannot hold one device
// twice).  Everything else -- shard bookkeeping, per-device seeds, root sum
// and check on the first context, short / empty shard padding -- is the
// production code path, so a one-GPU box executes the D >= 2 branches.

namespace {

struct rccl_api {
  void* h = nullptr;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

int load_rccl(rccl_api& r) {
  const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
  for (const char* nm : names) {
    r.h = dlopen(nm, RTLD_NOW | RTLD_LOCAL);
    if (r.h) break;
  }
  if (!r.h) return set_err(DGPU_EUNSUPPORTED, "RCCL not found (dlopen librccl.so.1: %s)", dlerror());
  r.comm_init_all = (decltype(r.comm_init_all))dlsym(r.h, "ncclCommInitAll");
  r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
  r.all_gather = (decltype(r.all_gather))dlsym(r.h, "ncclAllGather");
  r.group_start = (decltype(r.group_start))dlsym(r.h, "ncclGroupStart");
  r.group_end = (decltype(r.group_end))dlsym(r.h, "ncclGroupEnd");
  r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
  if (!r.comm_init_all || !r.comm_destroy || !r.all_gather || !r.group_start || !r.group_end || !r.error_string)
    return set_err(DGPU_EUNSUPPORTED, "RCCL is missing a symbol");
  return DGPU_OK;
}

#define NCCL_TRY(api, expr)                                                                            \
  do {                                                                                                 \
    ncclResult_t _r = (expr);                                                                          \
    if (_r != ncclSuccess) return set_err(DGPU_EDEVICE, "%s: %s", #expr, (api).error_string(_r));    \
  } while (0)

// per-device buffers of the gathers
struct multi_bufs {
  DevBuf bits, reasons, all_bits, all_reasons, root, all_roots;
};

}  // namespace

struct dgpu_multi {
  int ndev = 0;
  std::vector<int> devs;
  std::vector<dgpu_ctx*> ctx;
  std::vector<ncclComm_t> comm;
  std::vector<multi_bufs> buf;
  rccl_api api;
  std::mutex mu;
  bool loopback = false;          // DGPU_MULTI_ALLOW_SAME_DEVICE=1: device copies instead of RCCL (tests)
  std::vector<hipEvent_t> gev;    // loopback: per-device "source ready" events
};

extern "C" {

int dgpu_multi_open(int ndev, const int* devs, dgpu_multi** out) {
  if (!out || !devs || ndev < 1) return set_err(DGPU_EINVAL, "bad arguments");
  *out = nullptr;
  const char* same = getenv("DGPU_MULTI_ALLOW_SAME_DEVICE");
  const bool loopback = same && !strcmp(same, "1");
  for (int i = 0; i < ndev && !loopback; ++i)
    for (int j = 0; j < i; ++j)
      if (devs[i] == devs[j]) return set_err(DGPU_EINVAL, "device %d listed twice", devs[i]);
  dgpu_multi* m = new dgpu_multi();
  m->loopback = loopback;
  int rc = loopback ? DGPU_OK : load_rccl(m->api);
  if (rc) {
    delete m;
    return rc;
  }
  m->ndev = ndev;
  m->devs.assign(devs, devs + ndev);
  m->buf.resize(ndev);
  for (int i = 0; i < ndev; ++i) {
    dgpu_ctx* c = nullptr;
    if ((rc = dgpu_open(devs[i], &c))) {
      std::string msg = g_last_error;
      dgpu_multi_close(m);
      return set_err(rc, "%s", msg.c_str());
    }
    m->ctx.push_back(c);
  }
  if (loopback) {
    m->gev.assign(ndev, nullptr);
    for (int i = 0; i < ndev; ++i) {
      hipSetDevice(devs[i]);
      if (hipEventCreateWithFlags(&m->gev[i], hipEventDisableTiming) != hipSuccess) {
        dgpu_multi_close(m);
        return set_err(DGPU_EDEVICE, "hipEventCreate failed");
      }
    }
    *out = m;
    return DGPU_OK;
  }
  m->comm.resize(ndev);
  ncclResult_t r = m->api.comm_init_all(m->comm.data(), ndev, devs);
  if (r != ncclSuccess) {
    std::string msg = m->api.error_string(r);
    m->comm.clear();
    dgpu_multi_close(m);
    return set_err(DGPU_EDEVICE, "ncclCommInitAll: %s", msg.c_str());
  }
  *out = m;
  return DGPU_OK;
}

void dgpu_multi_close(dgpu_multi* m) {
  if (!m) return;
  for (size_t i = 0; i < m->comm.size(); ++i)
    if (m->comm[i]) m->api.comm_destroy(m->comm[i]);
  for (size_t i = 0; i < m->ctx.size(); ++i) {
    hipSetDevice(m->devs[i]);
    for (DevBuf* b : {&m->buf[i].bits, &m->buf[i].reasons, &m->buf[i].all_bits, &m->buf[i].all_reasons,
                      &m->buf[i].root, &m->buf[i].all_roots})
      b->release();
    if (i < m->gev.size() && m->gev[i]) hipEventDestroy(m->gev[i]);
    dgpu_close(m->ctx[i]);
  }
  delete m;
}

int dgpu_multi_context(dgpu_multi* m, int k, dgpu_ctx** out) {
  if (!m || !out || k < 0 || k >= m->ndev) return set_err(DGPU_EINVAL, "bad arguments");
  *out = m->ctx[k];
  return DGPU_OK;
}

}  // extern "C"

namespace {

// Run fn(k) for every device on its own host thread; the first failure's
// code and message become this thread's.
template <class Fn>
int for_each_device(dgpu_multi* m, Fn&& fn) {
  std::vector<int> rcs(m->ndev, DGPU_OK);
  std::vector<std::string> errs(m->ndev);
  std::vector<std::thread> th;
  for (int k = 0; k < m->ndev; ++k)
    th.emplace_back([&, k]() {
      if (hipSetDevice(m->devs[k]) != hipSuccess) {
        rcs[k] = DGPU_EDEVICE;
        errs[k] = "hipSetDevice failed";
        return;
      }
      rcs[k] = fn(k);
      if (rcs[k]) errs[k] = g_last_error;
    });
  for (auto& t : th) t.join();
  for (int k = 0; k < m->ndev; ++k)
    if (rcs[k]) return set_err(rcs[k], "device %d: %s", m->devs[k], errs[k].c_str());
  return DGPU_OK;
}

// One all-gather per device of `bytes` bytes: dst[k] + j * bytes <- src[j]
// for every j, enqueued on each device's stream.  RCCL (one group) or, in
// loopback mode, device copies ordered after every source stream's event.
int multi_all_gather(dgpu_multi* m, const std::vector<const void*>& src, const std::vector<void*>& dst,
                     size_t bytes) {
  const int D = m->ndev;
  if (!m->loopback) {
    NCCL_TRY(m->api, m->api.group_start());
    for (int k = 0; k < D; ++k)
      NCCL_TRY(m->api, m->api.all_gather(src[k], dst[k], bytes, ncclUint8, m->comm[k], m->ctx[k]->stream));
    NCCL_TRY(m->api, m->api.group_end());
    return DGPU_OK;
  }
  for (int j = 0; j < D; ++j) {
    HIP_TRY(hipSetDevice(m->devs[j]));
    HIP_TRY(hipEventRecord(m->gev[j], m->ctx[j]->stream));
  }
  for (int k = 0; k < D; ++k) {
    HIP_TRY(hipSetDevice(m->devs[k]));
    for (int j = 0; j < D; ++j) {
      HIP_TRY(hipStreamWaitEvent(m->ctx[k]->stream, m->gev[j], 0));
      HIP_TRY(hipMemcpyAsync((uint8_t*)dst[k] + (size_t)j * bytes, src[j], bytes, hipMemcpyDeviceToDevice,
                             m->ctx[k]->stream));
    }
  }
  return DGPU_OK;
}

// status -> verdict bits / reasons of one device's shard
int pack_shard_locked(dgpu_ctx* c, size_t cnt, uint8_t* d_bits, uint8_t* d_reason, hipStream_t s) {
  if (cnt == 0) return DGPU_OK;
  hipLaunchKernelGGL(k_pack_verdicts, dim3(grid_for((cnt + 7) / 8, 256)), dim3(256), 0, s, cnt,
                     (const uint8_t*)c->status.p, d_bits);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(d_reason, c->status.p, cnt, hipMemcpyDeviceToDevice, s));
  return DGPU_OK;
}

}  // namespace

extern "C" {

int dgpu_verify_multi(dgpu_multi* m, int scheme, const uint8_t* pk, size_t pk_len, size_t n, const uint64_t* rounds,
                      const uint8_t* sigs, size_t sig_stride, const uint32_t* sig_len, const uint8_t* prev,
                      size_t prev_stride, const uint32_t* prev_len, int mode, uint64_t rlc_seed,
                      uint8_t* verdict_bits, uint8_t* reason) {
  if (!m) return set_err(DGPU_EINVAL, "null handle");
  if (n == 0) return DGPU_OK;
  if (!verdict_bits) return set_err(DGPU_EINVAL, "null verdict buffer");
  const bool chained = scheme == DGPU_SCHEME_CHAINED;
  std::lock_guard<std::mutex> mlk(m->mu);
  std::vector<std::unique_lock<std::mutex>> locks;
  for (dgpu_ctx* c : m->ctx) locks.emplace_back(c->mu);
  const int D = m->ndev;
  // per-device shard capacity (a multiple of 8 rounds; dgpu_shard_range's rule)
  const size_t per = (((n + (size_t)D - 1) / (size_t)D) + 7) & ~(size_t)7;
  std::vector<key_entry*> keys(D, nullptr);
  std::vector<verify_args> args(D);
  int rc;
  for (int k = 0; k < D; ++k) {
    dgpu_ctx* c = m->ctx[k];
    HIP_TRY(hipSetDevice(c->device));
    if ((rc = get_key_locked(c, scheme, pk, pk_len, &keys[k]))) return rc;
    size_t lo, hi;
    dgpu_shard_range(n, D, k, &lo, &hi);
    // RLC coefficients: an independent seed per device (positions restart at 0)
    args[k] = verify_args{scheme, hi - lo, beacon_src(rounds + lo, chained ? prev + lo * prev_stride : nullptr,
                                                      prev_stride, chained ? prev_len + lo : nullptr, chained),
                          sigs + lo * sig_stride, sig_stride, sig_len + lo, mode,
                          D > 1 ? splitmix_host(rlc_seed ^ (0x5EEDull * (uint64_t)(k + 1))) : rlc_seed};
    if ((rc = check_args(c, keys[k], args[k]))) return rc;
    multi_bufs& b = m->buf[k];
    if ((rc = b.bits.ensure(per / 8)) || (rc = b.reasons.ensure(per)) || (rc = b.all_bits.ensure(D * per / 8)) ||
        (rc = b.all_reasons.ensure(D * per)) || (rc = b.root.ensure(2 * G2J_WORDS * 4)) ||
        (rc = b.all_roots.ensure((size_t)D * 2 * G2J_WORDS * 4)))
      return rc;
    HIP_TRY(hipStreamWaitEvent(c->stream, c->done, 0));
  }
  const bool rlc = mode == DGPU_MODE_RLC;
  const bool g1 = sig_on_g1(scheme);
  const int jw = g1 ? G1J_WORDS : G2J_WORDS;  // root: P, S (stride-1 Jacobian of the signature group)
  // phase 1: stage the shard (the records of the device's shard through its
  // context's pinned ring, overlapped with the verification) and verify it
  // per round (or compute its RLC root)
  rc = for_each_device(m, [&](int k) -> int {
    dgpu_ctx* c = m->ctx[k];
    verify_args& a = args[k];
    if (a.n == 0) return DGPU_OK;
    hipStream_t s = c->stream;
    int r;
    if ((r = c->status.ensure(a.n))) return r;
    c->n_ev = 0;
    c->ev_overflow = false;
    if (rlc) {  // the shard's points and its root by bucket MSM (the leaves wait for a failing root)
      c->rlc_pending = false;  // overwrites the points a pending per-rank root (dgpu_rlc_root_device) kept
      if ((r = stage_all_host_locked(c, a, s)) || (r = rlc_points_locked(c, a, s)) ||
          (r = c->msm_root.ensure(2 * (size_t)jw * 4)))
        return r;
      return rlc_root_msm_locked(c, a, s, (uint32_t*)c->msm_root.p);
    }
    // the shard's records through the context's pinned ring, slice by slice
    // beside the verification (verify_status_host_locked)
    if ((r = verify_status_host_locked(c, keys[k], a, s))) return r;
    return pack_shard_locked(c, a.n, (uint8_t*)m->buf[k].bits.p, (uint8_t*)m->buf[k].reasons.p, s);
  });
  if (rc) return rc;
  if (rlc) {
    bool all_ok = false;
    {
      // the per-device roots to every device; one check of their sum on device 0
      // the identity (Z = 0) of the signature group, for empty shards
      uint32_t inf_words[G2J_WORDS];
      rlc_identity_words(g1, inf_words);
      for (int k = 0; k < D; ++k) {
        dgpu_ctx* c = m->ctx[k];
        HIP_TRY(hipSetDevice(c->device));
        uint32_t* root = (uint32_t*)m->buf[k].root.p;
        if (args[k].n == 0) {
          HIP_TRY(hipMemcpyAsync(root, inf_words, (size_t)jw * 4, hipMemcpyHostToDevice, c->stream));
          HIP_TRY(hipMemcpyAsync(root + jw, inf_words, (size_t)jw * 4, hipMemcpyHostToDevice, c->stream));
        } else {
          HIP_TRY(hipMemcpyAsync(root, c->msm_root.p, 2 * (size_t)jw * 4, hipMemcpyDeviceToDevice, c->stream));
        }
      }
      std::vector<const void*> src(D);
      std::vector<void*> dst(D);
      for (int k = 0; k < D; ++k) {
        src[k] = m->buf[k].root.p;
        dst[k] = m->buf[k].all_roots.p;
      }
      if ((rc = multi_all_gather(m, src, dst, 2 * (size_t)jw * 4))) return rc;
      dgpu_ctx* c0 = m->ctx[0];
      HIP_TRY(hipSetDevice(c0->device));
      if ((rc = c0->rlc_root.ensure(2 * (size_t)jw * 4))) return rc;
      uint32_t* sum = (uint32_t*)c0->rlc_root.p;
      if (g1)
        hipLaunchKernelGGL(k_rlc_sum_roots<G1Ops>, dim3(1), dim3(64), 0, c0->stream, D,
                           (const uint32_t*)m->buf[0].all_roots.p, sum, sum + jw);
      else
        hipLaunchKernelGGL(k_rlc_sum_roots<G2Ops>, dim3(1), dim3(64), 0, c0->stream, D,
                           (const uint32_t*)m->buf[0].all_roots.p, sum, sum + jw);
      HIP_TRY(hipGetLastError());
      std::vector<uint8_t> fail;
      if ((rc = rlc_check_locked(c0, keys[0], std::vector<uint32_t>{0}, 1, sum, sum + jw, c0->stream, &fail)))
        return rc;
      all_ok = !fail[0];
    }
    rc = for_each_device(m, [&](int k) -> int {
      dgpu_ctx* c = m->ctx[k];
      const size_t cnt = args[k].n;
      if (cnt == 0) return DGPU_OK;
      int r;
      // this shard's verdicts, its own root first (D = 1: that root is the node's, known failing)
      if (!all_ok && (r = rlc_resolve_locked(c, keys[k], args[k], c->stream, (const uint32_t*)c->msm_root.p, D == 1)))
        return r;
      return pack_shard_locked(c, cnt, (uint8_t*)m->buf[k].bits.p, (uint8_t*)m->buf[k].reasons.p, c->stream);
    });
    if (rc) return rc;
  }
  // the verdicts of every shard to every device (one grouped all-gather)
  for (int k = 0; k < D; ++k) {
    HIP_TRY(hipSetDevice(m->ctx[k]->device));
    if (args[k].n < per) {  // padding of a short (or empty) last shard
      const size_t b0 = (args[k].n + 7) / 8;
      HIP_TRY(hipMemsetAsync((uint8_t*)m->buf[k].bits.p + b0, 0, per / 8 - b0, m->ctx[k]->stream));
    }
  }
  {
    std::vector<const void*> src(D), rsrc(D);
    std::vector<void*> dst(D), rdst(D);
    for (int k = 0; k < D; ++k) {
      src[k] = m->buf[k].bits.p;
      dst[k] = m->buf[k].all_bits.p;
      rsrc[k] = m->buf[k].reasons.p;
      rdst[k] = m->buf[k].all_reasons.p;
    }
    if ((rc = multi_all_gather(m, src, dst, per / 8))) return rc;
    if (reason && (rc = multi_all_gather(m, rsrc, rdst, per))) return rc;
  }
  for (int k = 0; k < D; ++k) {
    HIP_TRY(hipSetDevice(m->ctx[k]->device));
    HIP_TRY(hipStreamSynchronize(m->ctx[k]->stream));
  }
  dgpu_ctx* c0 = m->ctx[0];
  HIP_TRY(hipSetDevice(c0->device));
  HIP_TRY(hipMemcpyAsync(verdict_bits, m->buf[0].all_bits.p, (n + 7) / 8, hipMemcpyDeviceToHost, c0->stream));
  if (reason) HIP_TRY(hipMemcpyAsync(reason, m->buf[0].all_reasons.p, n, hipMemcpyDeviceToHost, c0->stream));
  for (int k = 0; k < D; ++k) {
    HIP_TRY(hipSetDevice(m->ctx[k]->device));
    HIP_TRY(hipEventRecord(m->ctx[k]->done, m->ctx[k]->stream));
    HIP_TRY(hipStreamSynchronize(m->ctx[k]->stream));
  }
  return DGPU_OK;
}

}  // extern "C"

extern "C" {

int dgpu_multi_set_group(dgpu_multi* m, int t, int n, const uint8_t* commits48) {
  if (!m) return set_err(DGPU_EINVAL, "null handle");
  std::lock_guard<std::mutex> mlk(m->mu);
  for (int k = 0; k < m->ndev; ++k) {
    int rc = dgpu_set_group(m->ctx[k], t, n, commits48);
    if (rc) return set_err(rc, "device %d: %s", m->devs[k], std::string(g_last_error).c_str());
  }
  return DGPU_OK;
}

// Threshold recovery over the node: rounds shard contiguously like the verify
// batch (dgpu_shard_range); each device stages and recovers its shard
// (recover_device_locked: VerifyPartial / selection / Lagrange + MSM /
// VerifyRecovered), the per-device recovery bitmaps are all-gathered (RCCL),
// and the recovered signatures and per-partial statuses -- data, not
// verdicts -- go to the host straight from the device that made them.
int dgpu_recover_multi(dgpu_multi* m, size_t n_rounds, const uint8_t* msgs32, size_t m_slots, const uint8_t* partials,
                       size_t partial_stride, const uint32_t* partial_len, uint8_t* out_sigs96, uint8_t* ok_bits,
                       uint8_t* partial_valid) {
  if (!m) return set_err(DGPU_EINVAL, "null multi handle");
  if (n_rounds == 0) return DGPU_OK;  // an empty batch: no-op, NULL buffers accepted
  if (!msgs32 || !partials || !partial_len || !out_sigs96 || !ok_bits) return set_err(DGPU_EINVAL, "null argument");
  if (m_slots == 0 || partial_stride < 98) return set_err(DGPU_EINVAL, "need m >= 1 partial slots and stride >= 98");
  const size_t items = n_rounds * m_slots;
  for (size_t i = 0; i < items; ++i)
    if (partial_len[i] > partial_stride) return set_err(DGPU_EINVAL, "partial_len[%zu] > stride", i);
  std::lock_guard<std::mutex> mlk(m->mu);
  std::vector<std::unique_lock<std::mutex>> locks;
  for (dgpu_ctx* c : m->ctx) locks.emplace_back(c->mu);
  const int D = m->ndev;
  const size_t per = (((n_rounds + (size_t)D - 1) / (size_t)D) + 7) & ~(size_t)7;
  std::vector<size_t> lo(D), hi(D);
  int rc;
  for (int k = 0; k < D; ++k) {
    dgpu_ctx* c = m->ctx[k];
    if (!c->grp_t) return set_err(DGPU_ENOKEY, "device %d: no threshold group installed (dgpu_multi_set_group)",
                                  m->devs[k]);
    dgpu_shard_range(n_rounds, D, k, &lo[k], &hi[k]);
    HIP_TRY(hipSetDevice(c->device));
    multi_bufs& b = m->buf[k];
    if ((rc = b.bits.ensure(per / 8)) || (rc = b.all_bits.ensure(D * per / 8))) return rc;
    HIP_TRY(hipStreamWaitEvent(c->stream, c->done, 0));
  }
  std::vector<std::vector<uint8_t>> stv(D);
  rc = for_each_device(m, [&](int k) -> int {
    dgpu_ctx* c = m->ctx[k];
    hipStream_t s = c->stream;
    const size_t nr = hi[k] - lo[k], it = nr * m_slots;
    int r;
    if (nr == 0) {
      HIP_TRY(hipMemsetAsync(m->buf[k].bits.p, 0, per / 8, s));
      return DGPU_OK;
    }
    if ((r = c->rec_msgs.ensure(nr * 32)) || (r = c->rec_parts.ensure(it * partial_stride)) ||
        (r = c->rec_plen.ensure(it * 4)) || (r = c->rec_out.ensure(nr * 96)) || (r = c->rec_ok.ensure(nr)) ||
        (r = c->out_reason.ensure(it)))
      return r;
    HIP_TRY(hipMemcpyAsync(c->rec_msgs.p, msgs32 + lo[k] * 32, nr * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->rec_parts.p, partials + lo[k] * m_slots * partial_stride, it * partial_stride,
                           hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->rec_plen.p, partial_len + lo[k] * m_slots, it * 4, hipMemcpyHostToDevice, s));
    if ((r = recover_device_locked(c, nr, (const uint8_t*)c->rec_msgs.p, m_slots, (const uint8_t*)c->rec_parts.p,
                                   partial_stride, (const uint32_t*)c->rec_plen.p, (uint8_t*)c->rec_out.p,
                                   (uint8_t*)c->rec_ok.p, partial_valid ? (uint8_t*)c->out_reason.p : nullptr, s)))
      return r;
    HIP_TRY(hipMemsetAsync(m->buf[k].bits.p, 0, per / 8, s));
    hipLaunchKernelGGL(k_pack_ok, dim3(grid_for((nr + 7) / 8, 256)), dim3(256), 0, s, nr, (const uint8_t*)c->rec_ok.p,
                       (uint8_t*)m->buf[k].bits.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out_sigs96 + lo[k] * 96, c->rec_out.p, nr * 96, hipMemcpyDeviceToHost, s));
    if (partial_valid) {
      stv[k].resize(it);
      HIP_TRY(hipMemcpyAsync(stv[k].data(), c->out_reason.p, it, hipMemcpyDeviceToHost, s));
    }
    return DGPU_OK;
  });
  if (rc) return rc;
  std::vector<const void*> src(D);
  std::vector<void*> dst(D);
  for (int k = 0; k < D; ++k) {
    src[k] = m->buf[k].bits.p;
    dst[k] = m->buf[k].all_bits.p;
  }
  if ((rc = multi_all_gather(m, src, dst, per / 8))) return rc;
  dgpu_ctx* c0 = m->ctx[0];
  HIP_TRY(hipSetDevice(c0->device));
  HIP_TRY(hipMemcpyAsync(ok_bits, m->buf[0].all_bits.p, (n_rounds + 7) / 8, hipMemcpyDeviceToHost, c0->stream));
  for (int k = 0; k < D; ++k) {
    HIP_TRY(hipSetDevice(m->ctx[k]->device));
    HIP_TRY(hipEventRecord(m->ctx[k]->done, m->ctx[k]->stream));
    HIP_TRY(hipStreamSynchronize(m->ctx[k]->stream));
  }
  if (partial_valid)
    for (int k = 0; k < D; ++k)
      for (size_t i = 0; i < stv[k].size(); ++i) partial_valid[lo[k] * m_slots + i] = stv[k][i] == ST_OK;
  return DGPU_OK;
}

}  // extern "C"
