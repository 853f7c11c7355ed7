// Host-side helpers and the ABI identity functions of libmrec.
#include "common.h"

#include <mutex>
#include <unordered_map>

namespace mrec {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

mrec_status launch_status(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return MREC_EHIP;
  }
  return MREC_OK;
}

// workspace layout records (common.h): address -> the last plan issued into it
namespace {
struct WsRecord {
  int layout;
  int64_t batch;
  int n_tables;
  bool padded;
  uint64_t seq;
};
std::mutex g_ws_mu;
std::unordered_map<uintptr_t, WsRecord> g_ws_records;
uint64_t g_ws_seq = 0;
constexpr size_t kWsRecordsMax = 1 << 14;
const char *layout_name(int layout) { return layout == kLayoutHash ? "hash" : "sorted"; }
}  // namespace

void ws_layout_record(const void *ws, int layout, int64_t batch, int n_tables, bool padded) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  if (g_ws_records.size() >= kWsRecordsMax &&
      g_ws_records.find(reinterpret_cast<uintptr_t>(ws)) == g_ws_records.end()) {
    auto oldest = g_ws_records.begin();  // (only a process with 16 k live workspaces gets here)
    for (auto it = g_ws_records.begin(); it != g_ws_records.end(); ++it)
      if (it->second.seq < oldest->second.seq) oldest = it;
    g_ws_records.erase(oldest);
  }
  g_ws_records[reinterpret_cast<uintptr_t>(ws)] = WsRecord{layout, batch, n_tables, padded, ++g_ws_seq};
}

mrec_status ws_layout_check(const void *ws, int layout, int64_t batch, int n_tables,
                            const char *who) {
  if (batch == 0) return MREC_OK;  // nothing is read
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws_records.find(reinterpret_cast<uintptr_t>(ws));
  if (it == g_ws_records.end()) {
    set_error(std::string(who) + ": no embedding-backward plan was issued into this workspace");
    return MREC_EINVAL;
  }
  const WsRecord &r = it->second;
  if (r.layout != layout || r.batch != batch || r.n_tables != n_tables) {
    set_error(std::string(who) + ": workspace layout mismatch: the plan wrote the " +
              layout_name(r.layout) + " layout for " + std::to_string(r.batch) + " entries x " +
              std::to_string(r.n_tables) + " tables" + (r.padded ? " (padded exchange view)" : "") +
              ", this apply reads the " + layout_name(layout) + " layout for " +
              std::to_string(batch) + " x " + std::to_string(n_tables) +
              (layout == kLayoutHash ? "" :
               " (a padded plan past MREC_BWD_HASH_MAX_BATCH entries takes the hash layout: "
               "apply it with mrec_emb_bwd_apply_given / _wire)"));
    return MREC_EINVAL;
  }
  return MREC_OK;
}

static bool pow2(int64_t x) { return x > 0 && (x & (x - 1)) == 0; }

mrec_status make_bank_args(const mrec_table_bank *bank, BankArgs *out, int *elem_bytes,
                           int *lanes_per_row) {
  MREC_CHECK_ARG(bank != nullptr, "bank is NULL");
  MREC_CHECK_ARG(bank->data != nullptr, "bank->data is NULL");
  MREC_CHECK_ARG(bank->row_offset != nullptr && bank->rows != nullptr,
                 "bank->row_offset/rows is NULL");
  MREC_CHECK_ARG(bank->n_tables >= 1 && bank->n_tables <= MREC_MAX_TABLES,
                 "n_tables out of [1, MREC_MAX_TABLES]");
  MREC_CHECK_ARG(bank->dtype == MREC_F32 || bank->dtype == MREC_BF16, "bank dtype must be F32/BF16");
  const int eb = bank->dtype == MREC_F32 ? 4 : 2;
  const int epl = 16 / eb;
  MREC_CHECK_ARG(bank->dim >= epl && bank->dim % epl == 0,
                 "dim must be a positive multiple of 16 bytes' worth of elements");
  MREC_CHECK_ARG(bank->row_stride >= bank->dim + (bank->has_w ? 1 : 0), "row_stride too small");
  const int64_t row_bytes = static_cast<int64_t>(bank->row_stride) * eb;
  MREC_CHECK_ARG(pow2(row_bytes) && row_bytes >= 16 && row_bytes <= 256,
                 "row_stride*elem_size must be a power of two in [16, 256] bytes");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(bank->data) & 15) == 0, "bank->data not 16B aligned");
  out->data = static_cast<char *>(bank->data);
  for (int f = 0; f < bank->n_tables; ++f) {
    MREC_CHECK_ARG(bank->row_offset[f] >= 0 && bank->rows[f] >= 0, "negative row_offset/rows");
    out->row_offset[f] = bank->row_offset[f];
    out->rows[f] = bank->rows[f];
  }
  for (int f = bank->n_tables; f < MREC_MAX_TABLES; ++f) out->row_offset[f] = out->rows[f] = 0;
  out->n_tables = bank->n_tables;
  out->dim = bank->dim;
  out->row_stride = bank->row_stride;
  out->has_w = bank->has_w ? 1 : 0;
  *elem_bytes = eb;
  *lanes_per_row = static_cast<int>(row_bytes / 16);
  out->lpr = *lanes_per_row;
  // a fused Adam bank: readers catch stale rows up (adam_current)
  out->adam = OptArgs{};
  if (bank->optim && bank->optim->kind == MREC_BWD_ADAM) {
    const mrec_status st = make_opt_args(bank, MREC_BWD_ADAM, &out->adam);
    if (st != MREC_OK) return st;
  }
  return MREC_OK;
}

// host: the fused optimizer of a mode >= MREC_BWD_ADAGRAD from bank->optim
mrec_status make_opt_args(const mrec_table_bank *bank, int mode, OptArgs *out) {
  *out = OptArgs{};
  if (mode <= MREC_BWD_SGD_SR) return MREC_OK;
  const mrec_optim *o = bank->optim;
  MREC_CHECK_ARG(o != nullptr, "fused optimizer mode without bank->optim");
  MREC_CHECK_ARG(o->state0 != nullptr, "optimizer state0 is NULL");
  const int64_t need = mrec_emb_optim_state_ld(bank->dim, bank->has_w);
  MREC_CHECK_ARG(mode == MREC_BWD_ROWWISE_ADAGRAD || (o->state_ld >= need && o->state_ld % 4 == 0),
                 "optimizer state_ld < mrec_emb_optim_state_ld or not a multiple of 4");
  MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(o->state0) & 15) == 0, "optimizer state not 16B aligned");
  if (mode == MREC_BWD_ADAM) {
    MREC_CHECK_ARG(o->state1 && o->row_step && o->d_t, "ADAM needs state1, row_step and d_t");
    MREC_CHECK_ARG((reinterpret_cast<uintptr_t>(o->state1) & 15) == 0, "optimizer state not 16B aligned");
    MREC_CHECK_ARG(o->beta1 >= 0.f && o->beta1 < 1.f && o->beta2 >= 0.f && o->beta2 < 1.f,
                   "betas must be in [0, 1)");
  }
  MREC_CHECK_ARG(o->eps >= 0.f, "eps < 0");
  out->kind = mode;
  out->lr = o->lr;
  out->eps = o->eps;
  out->beta1 = o->beta1;
  out->beta2 = o->beta2;
  out->wd = o->weight_decay;
  out->gscale = o->grad_scale;
  out->flags = o->flags;
  out->s0 = o->state0;
  out->s1 = o->state1;
  out->row_step = o->row_step;
  out->d_t = o->d_t;
  out->ld = o->state_ld;
  return MREC_OK;
}

mrec_status make_ids_args(const mrec_ids *ids, int n_tables, IdsArgs *out) {
  MREC_CHECK_ARG(ids != nullptr && ids->field_ptr != nullptr, "ids / ids->field_ptr is NULL");
  MREC_CHECK_ARG(ids->dtype == MREC_I32 || ids->dtype == MREC_I64, "ids dtype must be I32/I64");
  MREC_CHECK_ARG(ids->stride >= 1, "ids stride must be >= 1");
  for (int f = 0; f < n_tables; ++f) {
    MREC_CHECK_ARG(ids->field_ptr[f] != nullptr, "ids field pointer is NULL");
    out->ptr[f] = ids->field_ptr[f];
  }
  for (int f = n_tables; f < MREC_MAX_TABLES; ++f) out->ptr[f] = nullptr;
  MREC_CHECK_ARG(ids->chunk >= 0 && (ids->chunk == 0 || ids->chunk_stride >= ids->chunk),
                 "ids chunk / chunk_stride invalid");
  MREC_CHECK_ARG(ids->chunk == 0 || ids->stride == 1, "chunked ids need stride 1");
  out->stride = ids->stride;
  out->chunk = ids->chunk;
  out->chunk_stride = ids->chunk_stride;
  out->is64 = ids->dtype == MREC_I64 ? 1 : 0;
  out->pad_negative = ids->pad_negative ? 1 : 0;
  return MREC_OK;
}

static unsigned long long *g_kclock_buf = nullptr;
static int g_kclock_slots = 0, g_kclock_next = 0;

KClock kclock_take() {
  if (!g_kclock_buf || g_kclock_next >= g_kclock_slots) return KClock{nullptr, 0};
  return KClock{g_kclock_buf, g_kclock_next++};
}

}  // namespace mrec

extern "C" {

void mrec_kernel_clock(void *buf, int32_t n_slots) {
  mrec::g_kclock_buf = static_cast<unsigned long long *>(buf);
  mrec::g_kclock_slots = buf ? n_slots : 0;
  mrec::g_kclock_next = 0;
}

int32_t mrec_kernel_clock_used(void) { return mrec::g_kclock_next; }

int mrec_abi_version(void) { return MREC_ABI_VERSION; }

const char *mrec_last_error(void) { return mrec::g_last_error.c_str(); }

}  // extern "C"
