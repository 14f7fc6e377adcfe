#include "render.h"

#include <charconv>
#include <cmath>
#include <cstring>
#include <initializer_list>
#include <map>
#include <set>
#include <string_view>
#include <tuple>

namespace gpumon {

// ---------------------------------------------------------------------------------------------
// formatting helpers
// ---------------------------------------------------------------------------------------------
void append_double(double v, std::string* out) {
  if (std::isnan(v)) {
    out->append("NaN");
    return;
  }
  if (std::isinf(v)) {
    out->append(v > 0 ? "+Inf" : "-Inf");
    return;
  }
  char buf[64];
  // Integral values (the common case: %, MHz, bytes) print without exponent or fraction.
  if (v == std::floor(v) && std::fabs(v) < 9.007199254740992e15) {
    auto r = std::to_chars(buf, buf + sizeof buf, static_cast<long long>(v));
    out->append(buf, r.ptr);
    return;
  }
  auto r = std::to_chars(buf, buf + sizeof buf, v);
  out->append(buf, r.ptr);
}

void escape_label_value(std::string_view v, std::string* out) {
  // fast path: most values (ids, BDFs, sensor names, pod names) need no escaping
  bool plain = true;
  for (char c : v)
    if (c == '\\' || c == '"' || c == '\n') {
      plain = false;
      break;
    }
  if (plain) {
    out->append(v);
    return;
  }
  for (char c : v) {
    switch (c) {
      case '\\': out->append("\\\\"); break;
      case '"': out->append("\\\""); break;
      case '\n': out->append("\\n"); break;
      default: out->push_back(c);
    }
  }
}

void escape_influx_tag(const std::string& v, std::string* out) {
  if (v.empty()) {
    out->push_back('-');  // empty tag values are invalid in line protocol
    return;
  }
  for (char c : v) {
    if (c == ',' || c == ' ' || c == '=') out->push_back('\\');
    if (c == '\n') {
      out->append("\\n");
      continue;
    }
    out->push_back(c);
  }
}

void escape_influx_field_str(const std::string& v, std::string* out) {
  for (char c : v) {
    if (c == '"' || c == '\\') out->push_back('\\');
    if (c == '\n') {
      out->append("\\n");
      continue;
    }
    out->push_back(c);
  }
}

namespace {
// One pattern element at p against character c: advances *next past the element; false when c does
// not match. A malformed class ('[' without ']') matches a literal '['.
bool glob_one(const char* p, char c, const char** next) {
  if (*p == '?') {
    *next = p + 1;
    return true;
  }
  if (*p == '[') {
    const char* q = p + 1;
    const bool neg = *q == '!' || *q == '^';
    if (neg) ++q;
    bool hit = false;
    const char* first = q;
    while (*q && (*q != ']' || q == first)) {
      if (q[1] == '-' && q[2] && q[2] != ']') {
        if (static_cast<unsigned char>(c) >= static_cast<unsigned char>(q[0]) &&
            static_cast<unsigned char>(c) <= static_cast<unsigned char>(q[2]))
          hit = true;
        q += 3;
      } else {
        if (*q == c) hit = true;
        ++q;
      }
    }
    if (*q == ']') {
      *next = q + 1;
      return hit != neg;
    }
    *next = p + 1;  // no closing ']': literal
    return c == '[';
  }
  if (*p == '\\' && p[1]) {
    *next = p + 2;
    return p[1] == c;
  }
  *next = p + 1;
  return *p == c;
}
}  // namespace

bool glob_match(const char* p, const char* s) {
  const char* star = nullptr;  // pattern position after the last '*'
  const char* mark = nullptr;  // name position that '*' is currently absorbing up to
  while (*s) {
    const char* next = nullptr;
    if (*p == '*') {
      while (*p == '*') ++p;
      star = p;
      mark = s;
      continue;
    }
    if (*p && glob_one(p, *s, &next)) {
      p = next;
      ++s;
      continue;
    }
    if (!star) return false;
    p = star;  // let the last '*' absorb one more character and retry
    s = ++mark;
  }
  while (*p == '*') ++p;
  return *p == 0;
}

bool family_matches(const std::vector<std::string>& include, const std::vector<std::string>& exclude,
                    const char* name) {
  auto any = [name](const std::vector<std::string>& globs) {
    for (const auto& g : globs)
      if (glob_match(g.c_str(), name)) return true;
    return false;
  };
  if (!include.empty() && !any(include)) return false;
  return exclude.empty() || !any(exclude);
}

bool family_selected(const RenderInput& in, const char* name) {
  static const std::vector<std::string> kNone;
  return family_matches(in.metrics_include ? *in.metrics_include : kNone,
                        in.metrics_exclude ? *in.metrics_exclude : kNone, name);
}

void filter_exposition(const std::string& body, const std::vector<std::string>& include,
                       const std::vector<std::string>& exclude, std::string* out) {
  out->clear();
  out->reserve(body.size());
  bool keep = true;
  std::string name;
  size_t pos = 0;
  while (pos < body.size()) {
    size_t eol = body.find('\n', pos);
    const size_t end = eol == std::string::npos ? body.size() : eol + 1;
    if (body.compare(pos, 7, "# HELP ") == 0) {
      const size_t a = pos + 7;
      size_t b = a;
      while (b < end && body[b] != ' ' && body[b] != '\n') ++b;
      name.assign(body, a, b - a);
      keep = family_matches(include, exclude, name.c_str());
    }
    if (keep) out->append(body, pos, end - pos);
    pos = end;
  }
}

namespace {

using Labels = std::vector<std::pair<const char*, std::string>>;

// The input being rendered on this thread: every family checks the filter against it.
thread_local const RenderInput* t_render_in = nullptr;

bool selected(const char* name) { return !t_render_in || family_selected(*t_render_in, name); }

// A metric family whose header is dropped again if no sample line follows it; a family the
// filter deselects writes nothing at all.
class Family {
 public:
  Family(std::string* o, const char* name, const char* help, const char* type)
      : o_(o), name_(name), mark_(o->size()), on_(selected(name)) {  // name_: one strlen, not one per sample
    if (!on_) return;
    o_->append("# HELP ").append(name_).push_back(' ');
    o_->append(help).push_back('\n');
    o_->append("# TYPE ").append(name_).push_back(' ');
    o_->append(type).push_back('\n');
  }
  ~Family() {
    if (on_ && !any_) o_->resize(mark_);
  }
  // base: preformatted `k="v",...` (may be empty); extra: additional label pairs. A braced list
  // at the call site binds the initializer_list overload: no vector on the heap per sample (the
  // per-XCD and per-link families are most of an 8-GPU exposition's lines).
  void add(const std::string& base, const Labels& extra, double v, const char* suffix = nullptr) {
    add_impl(base, extra, v, suffix);
  }
  void add(const std::string& base, std::initializer_list<std::pair<const char*, std::string_view>> extra,
           double v, const char* suffix = nullptr) {
    add_impl(base, extra, v, suffix);
  }
  void add(const std::string& base, double v) { add_impl(base, Labels{}, v, nullptr); }

 private:
  template <class L>
  void add_impl(const std::string& base, const L& extra, double v, const char* suffix) {
    if (!on_ || std::isnan(v)) return;
    any_ = true;
    o_->append(name_);
    if (suffix) o_->append(suffix);
    if (!base.empty() || extra.size() != 0) {
      o_->push_back('{');
      o_->append(base);
      bool first = base.empty();
      for (const auto& kv : extra) {
        if (!first) o_->push_back(',');
        first = false;
        o_->append(kv.first).append("=\"");
        escape_label_value(kv.second, o_);
        o_->push_back('"');
      }
      o_->push_back('}');
    }
    o_->push_back(' ');
    append_double(v, o_);
    o_->push_back('\n');
  }

  std::string* o_;
  std::string_view name_;
  size_t mark_;
  bool on_;
  bool any_ = false;
};

std::string label_str(const Labels& l) {
  std::string s;
  bool first = true;
  for (const auto& kv : l) {
    if (!first) s.push_back(',');
    first = false;
    s.append(kv.first).append("=\"");
    escape_label_value(kv.second, &s);
    s.push_back('"');
  }
  return s;
}

void histogram(std::string* o, const char* name, const char* help, const HistSnapshot& h,
               const std::string& base) {
  if (!selected(name)) return;
  o->append("# HELP ").append(name).append(" ").append(help).append("\n");
  o->append("# TYPE ").append(name).append(" histogram\n");
  uint64_t cum = 0;
  for (size_t i = 0; i < h.bounds.size(); ++i) {
    cum += i < h.counts.size() ? h.counts[i] : 0;
    o->append(name).append("_bucket{");
    if (!base.empty()) o->append(base).push_back(',');
    o->append("le=\"");
    append_double(h.bounds[i], o);
    o->append("\"} ");
    append_double(static_cast<double>(cum), o);
    o->push_back('\n');
  }
  o->append(name).append("_bucket{");
  if (!base.empty()) o->append(base).push_back(',');
  o->append("le=\"+Inf\"} ");
  append_double(static_cast<double>(h.count), o);
  o->push_back('\n');
  o->append(name).append("_sum");
  if (!base.empty()) o->append("{").append(base).append("}");
  o->push_back(' ');
  append_double(h.sum, o);
  o->push_back('\n');
  o->append(name).append("_count");
  if (!base.empty()) o->append("{").append(base).append("}");
  o->push_back(' ');
  append_double(static_cast<double>(h.count), o);
  o->push_back('\n');
}

const double kMiB = 1048576.0;

}  // namespace

void render_prometheus(const RenderInput& in, std::string* o) {
  struct Scope {  // the filter applies to this call only (renders may nest on no other path)
    explicit Scope(const RenderInput* in) { t_render_in = in; }
    ~Scope() { t_render_in = nullptr; }
  } scope(&in);
  const auto& st = *in.statics;
  const auto& sm = *in.samples;
  const size_t n = std::min(st.size(), sm.size());
  std::vector<std::string> dl(n);
  for (size_t d = 0; d < n; ++d)
    dl[d] = in.full_device_labels
                ? label_str({{"host", in.host}, {"gpu_id", st[d].gpu_id}, {"gpu_uuid", st[d].uuid},
                             {"bdf", st[d].bdf}})
                : label_str({{"host", in.host}, {"gpu_id", st[d].gpu_id}});
  auto devf = [&](const char* name, const char* help, const char* type, auto get) {
    Family f(o, name, help, type);
    for (size_t d = 0; d < n; ++d)
      if (sm[d].ok) f.add(dl[d], get(d));
  };
  const DeviceRates kNoRates;
  auto rate = [&](size_t d) -> const DeviceRates& {
    return (in.rates && d < in.rates->size()) ? (*in.rates)[d] : kNoRates;
  };

  // ---------------- node_gpu (reference measurement, gpu.py:136-143) ----------------
  if (in.compat_families) {
    devf("node_gpu_gpu_util", "GPU (gfx) utilization in percent. Reference node_gpu.gpu_util.",
         "gauge", [&](size_t d) { return sm[d].v[F_GFX_UTIL]; });
    devf("node_gpu_mem_util", "VRAM used / total in percent. Reference node_gpu.mem_util.", "gauge",
         [&](size_t d) {
           double u = sm[d].v[F_VRAM_USED], t = sm[d].v[F_VRAM_TOTAL];
           return (has(u) && has(t) && t > 0) ? u * 100.0 / t : kNaN;  // Q9 guard
         });
    devf("node_gpu_mem_used", "VRAM used in MiB. Reference node_gpu.mem_used.", "gauge",
         [&](size_t d) { return std::floor(sm[d].v[F_VRAM_USED] / kMiB); });
    devf("node_gpu_mem_total", "VRAM total in MiB. Reference node_gpu.mem_total.", "gauge",
         [&](size_t d) { return std::floor(sm[d].v[F_VRAM_TOTAL] / kMiB); });
    devf("node_gpu_mem_free", "VRAM free in MiB. Reference node_gpu.mem_free.", "gauge",
         [&](size_t d) {
           double u = sm[d].v[F_VRAM_USED], t = sm[d].v[F_VRAM_TOTAL];
           return (has(u) && has(t)) ? std::floor((t - u) / kMiB) : kNaN;
         });
    devf("node_gpu_mem_bw_util",
         "Memory controller (UMC/HBM) activity in percent (reference queried utilization.memory but "
         "dropped it).",
         "gauge", [&](size_t d) { return sm[d].v[F_UMC_UTIL]; });
  }

  // ---------------- MI355X extras ----------------
  if (in.extended_families) {
    {
      Family f(o, "gpu_up", "1 if the last sample of this GPU succeeded.", "gauge");
      for (size_t d = 0; d < n; ++d) f.add(dl[d], sm[d].ok ? 1.0 : 0.0);
    }
    {
      Family f(o, "gpu_info", "Static GPU identity (value is always 1).", "gauge");
      for (size_t d = 0; d < n; ++d) {
        Labels extra;
        if (!in.full_device_labels) {
          extra.emplace_back("gpu_uuid", st[d].uuid);
          extra.emplace_back("bdf", st[d].bdf);
        }
        for (auto& kv : Labels{{"model", st[d].model},
               {"serial", st[d].serial},
               {"gfx_target", st[d].gfx_target},
               {"hip_id", std::to_string(st[d].hip_id)},
               {"drm_card", std::to_string(st[d].drm_card)},
               {"compute_partition", st[d].compute_partition},
               {"memory_partition", st[d].memory_partition},
               {"driver_version", st[d].driver_version},
               {"driver_source", st[d].driver_source}})
          extra.push_back(std::move(kv));
        f.add(dl[d], extra, 1.0);
      }
    }
    devf("gpu_sample_fresh", "1 if the firmware metrics table advanced since the previous tick.",
         "gauge", [&](size_t d) { return sm[d].fresh ? 1.0 : 0.0; });
    devf("gpu_vram_used_bytes", "VRAM (HBM3E) used in bytes.", "gauge",
         [&](size_t d) { return sm[d].v[F_VRAM_USED]; });
    devf("gpu_vram_total_bytes", "VRAM (HBM3E) total in bytes.", "gauge",
         [&](size_t d) { return sm[d].v[F_VRAM_TOTAL]; });
    devf("gpu_gtt_used_bytes", "GTT (host-mapped) memory used in bytes.", "gauge",
         [&](size_t d) { return sm[d].v[F_GTT_USED]; });
    devf("gpu_mm_activity_percent", "Multimedia engine activity in percent.", "gauge",
         [&](size_t d) { return sm[d].v[F_MM_UTIL]; });
    devf("gpu_gfx_activity_avg_percent",
         "GFX activity averaged over the sampling interval (firmware accumulator).", "gauge",
         [&](size_t d) { return rate(d).gfx_activity_avg_pct; });
    devf("gpu_umc_activity_avg_percent",
         "Memory activity averaged over the sampling interval (firmware accumulator).", "gauge",
         [&](size_t d) { return rate(d).mem_activity_avg_pct; });
    {
      Family f(o, "gpu_temperature_celsius", "Temperature in degrees Celsius by sensor.", "gauge");
      static const std::pair<Field, const char*> kT[] = {
          {F_TEMP_EDGE, "edge"},   {F_TEMP_HOTSPOT, "hotspot"}, {F_TEMP_MEM, "mem"},
          {F_TEMP_VRGFX, "vrgfx"}, {F_TEMP_VRSOC, "vrsoc"},     {F_TEMP_VRMEM, "vrmem"}};
      for (size_t d = 0; d < n; ++d) {
        if (!sm[d].ok) continue;
        for (const auto& t : kT) f.add(dl[d], {{"sensor", t.second}}, sm[d].v[t.first]);
        for (int k = 0; k < kMaxHbm; ++k)
          f.add(dl[d], {{"sensor", "hbm" + std::to_string(k)}}, sm[d].hbm_temp[k]);
      }
    }
    devf("gpu_power_watts", "Current socket power in watts.", "gauge",
         [&](size_t d) { return sm[d].v[F_POWER_CUR]; });
    devf("gpu_power_average_watts", "Firmware-averaged socket power in watts.", "gauge",
         [&](size_t d) { return sm[d].v[F_POWER_AVG]; });
    devf("gpu_power_interval_watts",
         "Socket power averaged over the sampling interval from the energy accumulator.", "gauge",
         [&](size_t d) { return rate(d).power_from_energy_w; });
    devf("gpu_power_limit_watts", "Socket power cap in watts.", "gauge",
         [&](size_t d) { return sm[d].v[F_POWER_LIMIT]; });
    devf("gpu_energy_joules_total", "Energy consumed since driver load in joules.", "counter",
         [&](size_t d) { return sm[d].v[F_ENERGY_J]; });
    {
      Family f(o, "gpu_clock_mhz", "Current clock frequency in MHz by clock domain.", "gauge");
      static const std::pair<Field, const char*> kC[] = {{F_GFXCLK_CUR, "gfx"},
                                                         {F_SOCCLK_CUR, "soc"},
                                                         {F_UCLK_CUR, "mem"},
                                                         {F_VCLK0_CUR, "vclk0"},
                                                         {F_DCLK0_CUR, "dclk0"}};
      for (size_t d = 0; d < n; ++d) {
        if (!sm[d].ok) continue;
        for (const auto& c : kC) f.add(dl[d], {{"clock", c.second}}, sm[d].v[c.first]);
        f.add(dl[d], {{"clock", "gfx_avg"}}, sm[d].v[F_GFXCLK_AVG]);
      }
    }
    {
      Family f(o, "gpu_xcd_clock_mhz", "Current gfx clock per XCD (XCC) in MHz.", "gauge");
      for (size_t d = 0; d < n; ++d)
        if (sm[d].ok)
          for (int k = 0; k < kMaxGfxClks; ++k)
            f.add(dl[d], {{"xcd", std::to_string(k)}}, sm[d].gfxclks[k]);
    }
    {
      Family f(o, "gpu_xcd_busy_percent", "Instantaneous GFX busy per XCD (XCC) in percent.",
               "gauge");
      for (size_t d = 0; d < n; ++d)
        if (sm[d].ok)
          for (int k = 0; k < sm[d].n_xcd; ++k)
            f.add(dl[d], {{"xcd", std::to_string(k)}}, sm[d].xcd_busy[k]);
    }
    {
      Family f(o, "gpu_xcd_busy_avg_percent",
               "GFX busy per XCD averaged over the sampling interval (firmware accumulator).",
               "gauge");
      for (size_t d = 0; d < n; ++d) {
        const auto& r = rate(d);
        if (sm[d].ok && r.valid)
          for (int k = 0; k < r.n_xcd; ++k)
            f.add(dl[d], {{"xcd", std::to_string(k)}}, r.xcd_busy_avg[k]);
      }
    }
    {
      // MI355X gpu_metrics v1.8 per-XCC residencies: is each XCD's clock being held down, and why?
      Family f(o, "gpu_xcd_clock_below_limit_percent",
               "Share of the interval each XCD's clock was held below the host limit, by reason "
               "(ppt = power, thermal, any).",
               "gauge");
      for (size_t d = 0; d < n; ++d) {
        const auto& r = rate(d);
        if (!sm[d].ok || !r.valid || !r.has_xcd_limit) continue;
        for (int k = 0; k < r.n_xcd; ++k) {
          const std::string x = std::to_string(k);
          f.add(dl[d], {{"xcd", x}, {"reason", "ppt"}}, r.xcd_below_ppt_pct[k]);
          f.add(dl[d], {{"xcd", x}, {"reason", "thermal"}}, r.xcd_below_thm_pct[k]);
          f.add(dl[d], {{"xcd", x}, {"reason", "any"}}, r.xcd_below_total_pct[k]);
        }
      }
    }
    {
      Family f(o, "gpu_xcd_low_utilization_percent",
               "Share of the interval each XCD spent in the firmware's low-utilisation (power-down "
               "eligible) state; 0 while any process holds a compute context on the GPU.",
               "gauge");
      for (size_t d = 0; d < n; ++d) {
        const auto& r = rate(d);
        if (!sm[d].ok || !r.valid || !r.has_xcd_limit) continue;
        for (int k = 0; k < r.n_xcd; ++k) f.add(dl[d], {{"xcd", std::to_string(k)}}, r.xcd_low_util_pct[k]);
      }
    }
    devf("gpu_throttle_status", "Firmware throttle status bitfield.", "gauge",
         [&](size_t d) { return sm[d].v[F_THROTTLE_STATUS]; });
    {
      Family f(o, "gpu_violation_percent",
               "Share of the interval spent in a power/thermal limit (PVIOL/TVIOL).", "gauge");
      for (size_t d = 0; d < n; ++d) {
        const auto& r = rate(d);
        if (!sm[d].ok || !r.valid) continue;
        f.add(dl[d], {{"kind", "ppt"}}, r.ppt_violation_pct);
        f.add(dl[d], {{"kind", "socket_thermal"}}, r.thermal_violation_pct);
        f.add(dl[d], {{"kind", "prochot"}}, r.prochot_violation_pct);
        f.add(dl[d], {{"kind", "vr_thermal"}}, r.vr_thm_violation_pct);
        f.add(dl[d], {{"kind", "hbm_thermal"}}, r.hbm_thm_violation_pct);
      }
    }
    devf("gpu_fan_rpm", "Fan speed in RPM.", "gauge", [&](size_t d) { return sm[d].v[F_FAN_RPM]; });
    devf("gpu_pcie_link_width", "PCIe link width in lanes.", "gauge",
         [&](size_t d) { return sm[d].v[F_PCIE_WIDTH]; });
    devf("gpu_pcie_link_speed_gts", "PCIe link speed in GT/s.", "gauge",
         [&](size_t d) { return sm[d].v[F_PCIE_SPEED_GTS]; });
    devf("gpu_pcie_bandwidth_bytes_per_second",
         "PCIe bandwidth averaged over the sampling interval, both directions, in bytes/s: firmware "
         "pcie_bandwidth_acc over its 1 kHz accumulation ticks x pcie_bw_unit_bytes (102400 B/s per "
         "firmware unit, measured on MI355X against pinned host<->device copies: h2d within 0.4 %, d2h 5 % under).",
         "gauge", [&](size_t d) { return rate(d).pcie_Bps; });
    devf("gpu_pcie_bandwidth_inst_bytes_per_second",
         "Instantaneous PCIe bandwidth (firmware, the last 1 ms accumulation tick), both directions, in bytes/s "
         "(same unit as gpu_pcie_bandwidth_bytes_per_second).",
         "gauge", [&](size_t d) { return sm[d].v[F_PCIE_BW_INST]; });
    devf("gpu_pcie_replay_total", "PCIe replay count.", "counter",
         [&](size_t d) { return sm[d].v[F_PCIE_REPLAY]; });
    devf("gpu_pcie_recovery_total", "PCIe L0-to-recovery transitions.", "counter",
         [&](size_t d) { return sm[d].v[F_PCIE_L0_RECOV]; });
    {
      Family f(o, "gpu_voltage_volts", "Rail voltage in volts.", "gauge");
      for (size_t d = 0; d < n; ++d) {
        if (!sm[d].ok) continue;
        f.add(dl[d], {{"rail", "soc"}}, sm[d].v[F_VOLT_SOC]);
        f.add(dl[d], {{"rail", "gfx"}}, sm[d].v[F_VOLT_GFX]);
        f.add(dl[d], {{"rail", "mem"}}, sm[d].v[F_VOLT_MEM]);
      }
    }
    devf("gpu_vram_max_bandwidth_bytes_per_second", "HBM peak bandwidth at max memory clock.",
         "gauge", [&](size_t d) {
           double g = sm[d].v[F_VRAM_MAX_BW];
           return has(g) ? g * 1e9 : kNaN;
         });
    devf("gpu_cu_occupancy_percent",
         "Resident waves of every process as a share of the GPU's wave slots, in percent (KFD cu_occupancy = "
         "waves / max waves per CU, summed over processes, interval mean of occ_samples reads, capped at 100; "
         "the per-process split is pod_gpu_proc_cu_occupancy_percent).",
         "gauge", [&](size_t d) {
           const double cu = sm[d].v[F_CU_OCC];
           const int n_cu = st[d].num_cu;
           return has(cu) && n_cu > 0 ? std::min(100.0, 100.0 * cu / n_cu) : kNaN;
         });
    // ---- RAS / ECC (ras.h; the reference exports no health data) ----
    {
      Family f(o, "gpu_ecc_errors_total",
               "Accumulated RAS error count by block and type (uncorrectable / correctable / deferred).",
               "counter");
      for (size_t d = 0; d < n; ++d) {
        if (!sm[d].ok || !sm[d].ras.valid) continue;
        for (const auto& c : sm[d].ras.blocks) {
          f.add(dl[d], {{"block", c.block}, {"type", "uncorrectable"}}, static_cast<double>(c.ue));
          f.add(dl[d], {{"block", c.block}, {"type", "correctable"}}, static_cast<double>(c.ce));
          if (c.has_de) f.add(dl[d], {{"block", c.block}, {"type", "deferred"}}, static_cast<double>(c.de));
        }
      }
    }
    {
      Family f(o, "gpu_ras_events_total", "RAS events by kind (fatal error, poison creation / consumption).",
               "counter");
      for (size_t d = 0; d < n; ++d) {
        const auto& r = sm[d].ras;
        if (!sm[d].ok || !r.valid) continue;
        f.add(dl[d], {{"event", "fatal"}}, r.fatal);
        f.add(dl[d], {{"event", "poison_creation"}}, r.poison_created);
        f.add(dl[d], {{"event", "poison_consumption"}}, r.poison_consumed);
      }
    }
    devf("gpu_retired_pages", "VRAM pages in the bad-page table (retired or pending retirement).", "gauge",
         [&](size_t d) { return sm[d].ras.valid ? sm[d].ras.bad_pages : kNaN; });
    // ---- xGMI (replaces the reference's absent NVLink fields) ----
    {
      Family fs(o, "gpu_xgmi_link_up", "xGMI link status (1 up, 0 down/disabled).", "gauge");
      for (size_t d = 0; d < n; ++d)
        if (sm[d].ok)
          for (int k = 0; k < sm[d].n_links; ++k) {
            const auto& L = sm[d].links[k];
            if (L.status < 0) continue;
            fs.add(dl[d], {{"link", std::to_string(k)}, {"peer_bdf", L.peer_bdf}},
                   L.status == 1 ? 1.0 : 0.0);
          }
    }
    auto link_acc = [&](const char* name, const char* help, bool rd) {
      Family f(o, name, help, "counter");
      for (size_t d = 0; d < n; ++d)
        if (sm[d].ok && sm[d].acc.valid)
          for (int k = 0; k < sm[d].acc.n_links_acc; ++k) {
            if (sm[d].links[k].status < 0) continue;
            double kb = static_cast<double>(rd ? sm[d].acc.xgmi_rd_kb[k] : sm[d].acc.xgmi_wr_kb[k]);
            f.add(dl[d], {{"link", std::to_string(k)}}, kb * 1024.0);
          }
    };
    link_acc("gpu_xgmi_read_bytes_total", "Bytes received over the xGMI link.", true);
    link_acc("gpu_xgmi_write_bytes_total", "Bytes sent over the xGMI link.", false);
    auto link_rate = [&](const char* name, const char* help, int which) {
      Family f(o, name, help, "gauge");
      for (size_t d = 0; d < n; ++d) {
        const auto& r = rate(d);
        if (!sm[d].ok || !r.valid) continue;
        for (int k = 0; k < r.n_links; ++k) {
          const auto& L = sm[d].links[k];
          if (L.status < 0) continue;
          double v = kNaN;
          if (which == 0) v = r.xgmi_rd_Bps[k];
          else if (which == 1) v = r.xgmi_wr_Bps[k];
          else if (has(L.max_bandwidth_gbps) && L.max_bandwidth_gbps > 0)
            v = (r.xgmi_rd_Bps[k] + r.xgmi_wr_Bps[k]) * 8.0 / (L.max_bandwidth_gbps * 1e9 * 2.0);
          f.add(dl[d], {{"link", std::to_string(k)}}, v);
        }
      }
    };
    link_rate("gpu_xgmi_read_bytes_per_second", "xGMI receive rate over the sampling interval.", 0);
    link_rate("gpu_xgmi_write_bytes_per_second", "xGMI send rate over the sampling interval.", 1);
    link_rate("gpu_xgmi_link_utilization_ratio",
              "(rx+tx)/(2*link max bandwidth) over the sampling interval.", 2);
    {
      Family f(o, "gpu_xgmi_link_max_bandwidth_bytes_per_second", "xGMI link max bandwidth.",
               "gauge");
      for (size_t d = 0; d < n; ++d)
        if (sm[d].ok)
          for (int k = 0; k < sm[d].n_links; ++k) {
            const auto& L = sm[d].links[k];
            if (L.status < 0 || !has(L.max_bandwidth_gbps)) continue;
            f.add(dl[d], {{"link", std::to_string(k)}}, L.max_bandwidth_gbps * 1e9 / 8.0);
          }
    }
    devf("gpu_xgmi_link_speed_gbps", "xGMI per-lane bit rate in Gb/s.", "gauge",
         [&](size_t d) { return sm[d].v[F_XGMI_LINK_SPEED]; });
    if (in.proc_counts) {
      Family f(o, "gpu_process_count", "GPU processes seen on this device.", "gauge");
      for (size_t d = 0; d < n && d < in.proc_counts->size(); ++d)
        f.add(dl[d], static_cast<double>((*in.proc_counts)[d]));
    }
  }

  // ---------------- pod_gpu (reference measurement, gpu.py:206-216 / 240-250) ----------------
  if (in.pod_rows) {
    const auto& rows = *in.pod_rows;
    std::vector<std::string> rl(rows.size());
    for (size_t r = 0; r < rows.size(); ++r) {
      const auto& p = rows[r];
      const DeviceStatic* s = p.dev < static_cast<int>(n) ? &st[p.dev] : nullptr;
      Labels l = {{"host", in.host},
                  {"namespace", p.pod_namespace},
                  {"gpu_id", s ? s->gpu_id : "-"},
                  {"containerid", p.containerid},
                  {"pid", p.pid},
                  {"user_name", p.user_name},
                  {"procressname", p.procname},  // sic: reference field name (gpu.py:209)
                  {"podname", p.pod_name},
                  {"container", p.container}};
      for (const auto& kv : p.extra_labels) l.emplace_back(kv.first.c_str(), kv.second);
      rl[r] = label_str(l);
    }
    if (in.compat_families) {
      Family fm(o, "pod_gpu_used_memory", "GPU memory used by the process in MiB (0 for idle rows).",
                "gauge");
      for (size_t r = 0; r < rows.size(); ++r)
        fm.add(rl[r], std::floor(rows[r].used_memory_bytes / kMiB));
    }
    if (in.compat_families) {
      Family fu(o, "pod_gpu_gpu_util",
                "Device-wide GPU utilization copied to each process row (reference semantics; 0 for "
                "idle rows).",
                "gauge");
      for (size_t r = 0; r < rows.size(); ++r) fu.add(rl[r], rows[r].gpu_util);
    }
    {
      Family f(o, "pod_gpu_mfma_util_percent",
               "Wall-time MFMA (matrix core) utilisation of the GPU while this process was the only one with "
               "waves resident (exclusive use: no other process's waves in the last 5 ticks and "
               "mfma_exclusive_window_s): the device's gpu_mfma_util_percent. Absent when the GPU was shared or "
               "PMC counting is off.",
               "gauge");
      for (size_t r = 0; r < rows.size(); ++r)
        if (has(rows[r].mfma_util)) f.add(rl[r], rows[r].mfma_util);
    }
    {
      Family f(o, "pod_gpu_used_memory_bytes", "GPU memory (VRAM) used by the process in bytes.",
               "gauge");
      for (size_t r = 0; r < rows.size(); ++r) f.add(rl[r], rows[r].used_memory_bytes);
    }
    {
      Family f(o, "pod_gpu_proc_gfx_util",
               "Per-process GPU busy percent over the sampling interval: DRM fdinfo gfx engine time when the "
               "process submits through the kernel (graphics); for HIP compute on KFD user queues, the share of "
               "the interval's cu_occupancy reads that found the process's waves resident. Processes resident "
               "at the same time each count that time: on a shared GPU the values may add up to over 100.",
               "gauge");
      for (size_t r = 0; r < rows.size(); ++r) f.add(rl[r], rows[r].proc_gfx_util);
    }
    {
      Family f(o, "pod_gpu_proc_cu_occupancy",
               "The process's resident waves in CU-equivalents (KFD cu_occupancy = waves / max waves per CU; "
               "interval mean of occ_samples reads).",
               "gauge");
      for (size_t r = 0; r < rows.size(); ++r) f.add(rl[r], rows[r].cu_occupancy);
    }
    {
      // Per-process wave occupancy: the process's resident waves / the device's wave slots (KFD
      // counts waves / max waves per CU; 243 of 256 on MI355X under the saturating bf16 burn,
      // 7.7 under a 64-workgroup load, profiles/r2_kfd_occupancy.md).
      Family f(o, "pod_gpu_proc_cu_occupancy_percent",
               "The process's resident waves as a share of the GPU's wave slots, in percent (interval mean).",
               "gauge");
      for (size_t r = 0; r < rows.size(); ++r) {
        const int dev = rows[r].dev;
        const int cus = dev >= 0 && dev < static_cast<int>(in.statics->size()) ? (*in.statics)[dev].num_cu : 0;
        if (cus > 0 && has(rows[r].cu_occupancy))
          f.add(rl[r], std::min(100.0, 100.0 * rows[r].cu_occupancy / cus));
      }
    }
    {
      // KFD's per-process queue list: 0 = a context that never submitted work to this GPU
      Family f(o, "pod_gpu_proc_queues",
               "Hardware (user-mode) queues the process holds on this GPU (KFD); 0 = a context that never "
               "submitted work here.",
               "gauge");
      for (size_t r = 0; r < rows.size(); ++r)
        if (!rows[r].idle && rows[r].queues >= 0) f.add(rl[r], static_cast<double>(rows[r].queues));
    }
    // One series per (pod, container, gpu): the allocation view behind the reference dashboard's
    // "GPUs per user" and "allocated / in use" panels.
    {
      struct Key {
        std::string ns, pod, container, cid, user;
        int dev;
        std::vector<std::pair<std::string, std::string>> extra;
        bool operator<(const Key& o) const {
          return std::tie(ns, pod, container, cid, user, dev, extra) <
                 std::tie(o.ns, o.pod, o.container, o.cid, o.user, o.dev, o.extra);
        }
      };
      std::map<Key, bool> alloc;  // -> active
      for (const auto& p : rows) {
        if (p.pod_name == "-" && p.containerid == "-") continue;  // host process
        Key k{p.pod_namespace, p.pod_name, p.container, p.containerid, p.user_name, p.dev, p.extra_labels};
        alloc[k] = alloc[k] || !p.idle;
      }
      std::set<int> devs_alloc, devs_active;
      {
        Family f(o, "pod_gpu_allocated",
                 "1 per (pod, container, GPU) holding a GPU; state=active|idle.", "gauge");
        for (const auto& [k, active] : alloc) {
          const DeviceStatic* s = k.dev < static_cast<int>(n) ? &st[k.dev] : nullptr;
          Labels l = {{"host", in.host},
                      {"namespace", k.ns},
                      {"podname", k.pod},
                      {"container", k.container},
                      {"containerid", k.cid},
                      {"user_name", k.user},
                      {"gpu_id", s ? s->gpu_id : "-"},
                      {"state", active ? "active" : "idle"}};
          for (const auto& kv : k.extra) l.emplace_back(kv.first.c_str(), kv.second);
          f.add(label_str(l), 1.0);
          devs_alloc.insert(k.dev);
          if (active) devs_active.insert(k.dev);
        }
      }
      Family g(o, "gpumon_gpus", "GPU counts on this node: total / allocated / allocated_idle / "
                                  "allocated_active (reference dashboard stat panels).",
               "gauge");
      std::string hl = label_str({{"host", in.host}});
      g.add(hl, {{"state", "total"}}, static_cast<double>(n));
      g.add(hl, {{"state", "allocated"}}, static_cast<double>(devs_alloc.size()));
      g.add(hl, {{"state", "allocated_active"}}, static_cast<double>(devs_active.size()));
      g.add(hl, {{"state", "allocated_idle"}},
            static_cast<double>(devs_alloc.size() - devs_active.size()));
    }
  }

  // ---------------- extras (probe kernel, PMC, plugins) ----------------
  if (in.extras && !in.extras->empty()) {
    std::map<std::string, std::vector<const ExtraSeries*>> byname;
    for (const auto& e : *in.extras) byname[e.name].push_back(&e);
    for (const auto& [name, vec] : byname) {
      Family f(o, name.c_str(), vec[0]->help.empty() ? name.c_str() : vec[0]->help.c_str(),
               vec[0]->type.c_str());
      for (const auto* e : vec) {
        std::string base = (e->dev >= 0 && e->dev < static_cast<int>(n))
                               ? dl[e->dev]
                               : label_str({{"host", in.host}});
        Labels extra;
        for (const auto& kv : e->labels) extra.emplace_back(kv.first.c_str(), kv.second);
        f.add(base, extra, e->value);
      }
    }
  }

  // ---------------- exporter self-metrics ----------------
  if (in.self) {
    const SelfStats& s = *in.self;
    std::string hl = label_str({{"host", in.host}});
    {
      Family f(o, "gpumon_build_info", "Exporter build and backend identity.", "gauge");
      f.add(hl, {{"version", s.version}, {"backend", s.backend}, {"backend_version", s.backend_version}},
            1.0);
    }
    {
      Family f(o, "gpumon_backend_up", "1 if the device backend is initialised.", "gauge");
      f.add(hl, s.backend_up ? 1.0 : 0.0);
    }
    if (s.fast_path_devices >= 0) {
      Family f(o, "gpumon_fast_path_devices",
               "GPUs whose per-tick values are read straight from sysfs/KFD instead of libamd_smi.", "gauge");
      f.add(hl, static_cast<double>(s.fast_path_devices));
    }
    {
      Family f(o, "gpumon_backend_reinits_total",
               "Backend re-initialisations after every GPU failed for several ticks.", "counter");
      f.add(hl, static_cast<double>(s.backend_reinits));
    }
    {
      Family f(o, "gpumon_sample_interval_seconds", "Configured sampling interval.", "gauge");
      f.add(hl, s.interval_s);
    }
    {
      Family f(o, "gpumon_ticks_total", "Sampler ticks completed.", "counter");
      f.add(hl, static_cast<double>(s.ticks));
    }
    {
      Family f(o, "gpumon_samples_total", "Device samples taken (one per GPU per tick).", "counter");
      f.add(hl, static_cast<double>(s.samples));
    }
    {
      Family f(o, "gpumon_stale_samples_total",
               "Device samples whose firmware table had not advanced since the previous tick.",
               "counter");
      f.add(hl, static_cast<double>(s.stale_samples));
    }
    {
      Family f(o, "gpumon_frozen_samples_total",
               "Stale device samples whose table had not advanced for longer than stale_hold_s: the SMU stopped "
               "refreshing it, and the interval rates were withheld.",
               "counter");
      f.add(hl, static_cast<double>(s.frozen_samples));
    }
    {
      Family f(o, "gpumon_hidden_gpu_contexts",
               "Processes with a GPU context but no VRAM and no resident waves in the last tick, left out of the "
               "pod_gpu rows (hide_empty_contexts).",
               "gauge");
      f.add(hl, static_cast<double>(s.hidden_contexts));
    }
    {
      Family f(o, "gpumon_hidden_peer_gpu_contexts",
               "GPU contexts of multi-GPU processes on GPUs they do not work on (no hardware queue there in "
               "KFD's per-process queue list, or at most peer_context_max_vram_mib of VRAM where that list is "
               "unreadable; no resident waves in the sharing window; a workload on another GPU: e.g. every "
               "torchrun rank opening all GPUs), left out of the pod_gpu rows and gpu_active_processes.",
               "gauge");
      f.add(hl, static_cast<double>(s.hidden_peer_contexts));
    }
    {
      Family f(o, "gpumon_sampler_rt_threads",
               "Sampler and device-worker threads running SCHED_FIFO (rt_priority > 0 and CAP_SYS_NICE).", "gauge");
      f.add(hl, static_cast<double>(s.rt_threads));
    }
    if (s.http_max_conns >= 0) {
      Family f(o, "gpumon_http_max_connections",
               "Connections the HTTP loops hold at most (per-loop cap x loops; the cap comes from RLIMIT_NOFILE "
               "with 256 fds kept for the sampler).",
               "gauge");
      f.add(hl, static_cast<double>(s.http_max_conns));
    }
    if (s.http_evicted >= 0) {
      Family f(o, "gpumon_http_connections_evicted_total",
               "Idle connections closed to make room for a new one at the server's connection cap (derived "
               "from RLIMIT_NOFILE): a connection flood.",
               "counter");
      f.add(hl, static_cast<double>(s.http_evicted));
    }
    if (s.http_tls_failures >= 0) {
      Family f(o, "gpumon_http_tls_handshake_failures_total",
               "/metrics over HTTPS (tls_cert_file): connections whose TLS handshake failed or did not finish "
               "within the header timeout -- a plain-HTTP scraper, a scraper that does not trust the "
               "certificate, or (mutual TLS) one whose client certificate did not verify.",
               "counter");
      f.add(hl, static_cast<double>(s.http_tls_failures));
    }
    if (s.http_tls_client_cert_refused >= 0) {
      Family f(o, "gpumon_http_tls_client_cert_refused_total",
               "Mutual TLS (tls_client_ca_file): /metrics requests refused with 403 because the connection "
               "presented no client certificate (the health endpoints answer such connections: the "
               "kubelet's probes send none).",
               "counter");
      f.add(hl, static_cast<double>(s.http_tls_client_cert_refused));
    }
    if (s.http_tls_failures >= 0) {
      {
        Family f(o, "gpumon_http_tls_cert_not_after_timestamp_seconds",
                 "Expiry (unix seconds) of the certificate /metrics is served with; rotated files are picked up "
                 "within 5 s (gpumon_http_tls_reloads_total).",
                 "gauge");
        if (s.http_tls_not_after > 0) f.add(hl, static_cast<double>(s.http_tls_not_after));
      }
      Family f(o, "gpumon_http_tls_reloads_total",
               "Changes of tls_cert_file / tls_key_file / tls_client_ca_file seen: result=ok swapped in for new "
               "connections, result=error did not load (the previous certificate stays in use).",
               "counter");
      f.add(hl, {{"result", "ok"}}, static_cast<double>(s.http_tls_reloads_ok));
      f.add(hl, {{"result", "error"}}, static_cast<double>(s.http_tls_reloads_failed));
    }
    if (s.http_auth_failures >= 0) {
      {
        Family f(o, "gpumon_http_auth_failures_total",
                 "/metrics requests refused with 401 (http_auth_token_file) by reason: missing (no Authorization "
                 "header: a scraper without credentials), scheme (not Bearer), token (not one of the file's: a "
                 "stale token after a rotation, or a guess).",
                 "counter");
        static const char* const kReason[3] = {"missing", "scheme", "token"};
        for (int i = 0; i < 3; ++i) f.add(hl, {{"reason", kReason[i]}}, static_cast<double>(s.http_auth_failures_by[i]));
      }
      Family f(o, "gpumon_http_auth_token_reloads_total",
               "Changes of http_auth_token_file seen: result=ok the new token is required from the next request, "
               "result=error not usable (the previous token stays in force).",
               "counter");
      f.add(hl, {{"result", "ok"}}, static_cast<double>(s.http_auth_reloads_ok));
      f.add(hl, {{"result", "error"}}, static_cast<double>(s.http_auth_reloads_failed));
    }
    if (s.http_rt_loops >= 0) {
      {
        Family f(o, "gpumon_http_rt_loops",
                 "HTTP event loops running SCHED_FIFO right now (http_rt_priority; a loop past its CPU budget "
                 "runs at normal priority until its 100 ms window ends).",
                 "gauge");
        f.add(hl, static_cast<double>(s.http_rt_loops));
      }
      {
        Family f(o, "gpumon_http_rt_demotions_total",
                 "Times an SCHED_FIFO HTTP loop used its CPU budget (http_rt_budget per 100 ms) and dropped to "
                 "normal scheduling for the rest of the window: a request flood.",
                 "counter");
        f.add(hl, static_cast<double>(s.http_rt_demotions));
      }
    }
    {
      Family f(o, "gpumon_occupancy_reads_total",
               "KFD cu_occupancy reads made between ticks by the device workers (occ_samples per tick).",
               "counter");
      f.add(hl, static_cast<double>(s.occupancy_reads));
    }
    {
      Family f(o, "gpumon_process_list_failures_total",
               "Process lists of a GPU that can list processes that failed (a transient library or KFD "
               "error); the GPU's last good list is kept for up to 3 ticks (gpu_process_list_held).",
               "counter");
      f.add(hl, static_cast<double>(s.process_list_failures));
    }
    {
      Family f(o, "gpumon_occupancy_scan_failures_total",
               "Device-worker KFD process listings that failed (retried after 1 s, doubling to 60 s; the known "
               "pids are re-read meanwhile).",
               "counter");
      f.add(hl, static_cast<double>(s.occupancy_scan_failures));
    }
    {
      Family f(o, "gpumon_tick_overruns_total", "Ticks that took longer than the interval.",
               "counter");
      f.add(hl, static_cast<double>(s.overruns));
    }
    {
      Family f(o, "gpumon_last_sample_timestamp_seconds", "Wall time of the last completed tick.",
               "gauge");
      f.add(hl, s.last_tick_wall_s);
    }
    {
      Family f(o, "gpumon_sample_errors_total", "Failed backend calls per GPU.", "counter");
      for (size_t d = 0; d < s.device_errors.size() && d < n; ++d)
        f.add(dl[d], static_cast<double>(s.device_errors[d]));
    }
    {
      Family f(o, "gpumon_device_timeouts_total",
               "Ticks in which a GPU's backend call exceeded device_timeout_s (hung call; exported as gpu_up 0).",
               "counter");
      for (size_t d = 0; d < s.device_timeouts.size() && d < n; ++d)
        f.add(dl[d], static_cast<double>(s.device_timeouts[d]));
    }
    histogram(o, "gpumon_sample_duration_seconds",
              "Time to sample all GPUs, attribute processes, render and publish one tick (gzip follows the publish).", s.sample_hist, hl);
    histogram(o, "gpumon_scrape_duration_seconds",
              "Server-side /metrics latency (request parsed -> response written).", s.scrape_hist, hl);
    {
      Family f(o, "gpumon_scrapes_total", "HTTP /metrics requests served.", "counter");
      f.add(hl, static_cast<double>(s.scrapes));
    }
    {
      Family f(o, "gpumon_http_connections", "Open HTTP connections.", "gauge");
      f.add(hl, static_cast<double>(s.http_connections));
    }
    {
      Family f(o, "gpumon_pods_attributed", "pod_gpu rows produced in the last tick.", "gauge");
      f.add(hl, static_cast<double>(s.pods_attributed));
    }
    {
      Family f(o, "gpumon_attribution_cache_total", "PID attribution cache lookups by result.",
               "counter");
      f.add(hl, {{"result", "hit"}}, static_cast<double>(s.attribution_cache_hits));
      f.add(hl, {{"result", "miss"}}, static_cast<double>(s.attribution_cache_misses));
    }
    {
      Family f(o, "gpumon_influx_push_total", "InfluxDB compat pushes by result.", "counter");
      if (s.influx_ok || s.influx_fail || s.influx_dropped) {
        f.add(hl, {{"result", "ok"}}, static_cast<double>(s.influx_ok));
        f.add(hl, {{"result", "error"}}, static_cast<double>(s.influx_fail));
        f.add(hl, {{"result", "dropped"}}, static_cast<double>(s.influx_dropped));
      }
    }
    {
      Family f(o, "gpumon_snapshot_compressions_total",
               "gzip compressions of the /metrics snapshot: eager (the tick thread, while most snapshots are "
               "scraped with gzip), predicted (the tick thread, for a periodic scraper's next scrape) or lazy "
               "(by the first gzip scrape of a snapshot).", "counter");
      if (s.gzip_eager || s.gzip_lazy || s.gzip_predicted) {
        f.add(hl, {{"mode", "eager"}}, static_cast<double>(s.gzip_eager));
        f.add(hl, {{"mode", "predicted"}}, static_cast<double>(s.gzip_predicted));
        f.add(hl, {{"mode", "lazy"}}, static_cast<double>(s.gzip_lazy));
      }
    }
    {
      Family f(o, "gpumon_snapshot_compressions_unused_total",
               "Eager snapshot compressions no scrape fetched before the next tick replaced the snapshot.",
               "counter");
      if (s.gzip_eager || s.gzip_predicted) f.add(hl, static_cast<double>(s.gzip_unused));
    }
    {
      Family f(o, "gpumon_influx_up",
               "1 if the last InfluxDB compat push succeeded, 0 if it failed or none completed yet (push configured).",
               "gauge");
      if (s.influx_enabled) f.add(hl, static_cast<double>(s.influx_up));
    }
    {
      Family f(o, "gpumon_influx_last_success_timestamp_seconds",
               "Unix time of the last successful InfluxDB compat push.", "gauge");
      if (s.influx_enabled && s.influx_last_ok_wall_ns > 0) f.add(hl, s.influx_last_ok_wall_ns * 1e-9);
    }
    {
      Family f(o, "process_cpu_seconds_total", "Exporter user+system CPU time.", "counter");
      if (s.cpu_seconds >= 0) f.add(hl, s.cpu_seconds);
    }
    {
      Family f(o, "process_resident_memory_bytes", "Exporter resident memory.", "gauge");
      if (s.rss_bytes >= 0) f.add(hl, s.rss_bytes);
    }
    {
      Family f(o, "process_start_time_seconds", "Exporter start time (unix seconds).", "gauge");
      if (s.start_time_s >= 0) f.add(hl, s.start_time_s);
    }
    {
      Family f(o, "process_threads", "Exporter OS threads.", "gauge");
      if (s.threads >= 0) f.add(hl, s.threads);
    }
    {
      Family f(o, "process_open_fds", "Exporter open file descriptors.", "gauge");
      if (s.open_fds >= 0) f.add(hl, s.open_fds);
    }
    {
      Family f(o, "gpumon_backend_calls_total", "Device-library calls by kind.", "counter");
      for (const auto& c : s.backend_calls) f.add(hl, {{"call", c.call}}, static_cast<double>(c.n));
    }
    {
      Family f(o, "gpumon_backend_call_seconds_total", "Time spent in device-library calls by kind.",
               "counter");
      for (const auto& c : s.backend_calls) f.add(hl, {{"call", c.call}}, c.seconds);
    }
    {
      Family f(o, "gpumon_backend_call_errors_total", "Failed device-library calls by kind.", "counter");
      for (const auto& c : s.backend_calls) f.add(hl, {{"call", c.call}}, static_cast<double>(c.errors));
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Influx line protocol (reference-compatible)
// ---------------------------------------------------------------------------------------------
void render_influx(const RenderInput& in, int64_t ts_ns, bool extended, std::string* o, int schema) {
  const auto& st = *in.statics;
  const auto& sm = *in.samples;
  const size_t n = std::min(st.size(), sm.size());
  auto num = [&](double v) { append_double(has(v) ? v : 0.0, o); };
  for (size_t d = 0; d < n; ++d) {
    if (!sm[d].ok) continue;
    const auto& v = sm[d].v;
    double used = std::floor(v[F_VRAM_USED] / kMiB), total = std::floor(v[F_VRAM_TOTAL] / kMiB);
    // node_gpu,host=H,gpu_id=K gpu_util=U,mem_util=F,mem_used=M,mem_total=T,node="H",gid=K,mem_free=F
    o->append("node_gpu,host=");
    escape_influx_tag(in.host, o);
    o->append(",gpu_id=");
    escape_influx_tag(st[d].gpu_id, o);
    o->append(" gpu_util=");
    num(v[F_GFX_UTIL]);
    o->append(",mem_util=");
    num(has(used) && total > 0 ? v[F_VRAM_USED] * 100.0 / v[F_VRAM_TOTAL] : 0.0);
    o->append(",mem_used=");
    num(used);
    o->append(",mem_total=");
    num(total);
    o->append(",node=\"");
    escape_influx_field_str(in.host, o);
    o->append("\",gid=");
    o->append(st[d].gpu_id);
    o->append(",mem_free=");
    num(total - used);
    o->push_back(' ');
    o->append(std::to_string(ts_ns));
    o->push_back('\n');
    if (extended) {
      o->append("gpu_ext,host=");
      escape_influx_tag(in.host, o);
      o->append(",gpu_id=");
      escape_influx_tag(st[d].gpu_id, o);
      o->append(",gpu_uuid=");
      escape_influx_tag(st[d].uuid, o);
      bool first = true;
      auto field = [&](const char* k, double x) {
        if (!has(x)) return;
        o->push_back(first ? ' ' : ',');
        first = false;
        o->append(k).push_back('=');
        append_double(x, o);
      };
      field("mem_bw_util", v[F_UMC_UTIL]);
      field("temp_hotspot", v[F_TEMP_HOTSPOT]);
      field("temp_mem", v[F_TEMP_MEM]);
      field("power_w", v[F_POWER_CUR]);
      field("energy_j", v[F_ENERGY_J]);
      field("gfxclk_mhz", v[F_GFXCLK_CUR]);
      field("uclk_mhz", v[F_UCLK_CUR]);
      if (in.rates && d < in.rates->size() && (*in.rates)[d].valid) {  // interval rates (rates.cpp)
        field("pcie_bytes_per_s", (*in.rates)[d].pcie_Bps);
        field("power_interval_w", (*in.rates)[d].power_from_energy_w);
      }
      for (int k = 0; k < sm[d].n_xcd; ++k) {
        std::string key = "xcd" + std::to_string(k) + "_busy";
        field(key.c_str(), sm[d].xcd_busy[k]);
      }
      if (sm[d].ras.valid) {  // RAS totals over every block (ras.h)
        double ue = 0, ce = 0;
        for (const auto& c : sm[d].ras.blocks) {
          ue += static_cast<double>(c.ue);
          ce += static_cast<double>(c.ce);
        }
        field("ecc_uncorrectable", ue);
        field("ecc_correctable", ce);
        field("retired_pages", sm[d].ras.bad_pages);
      }
      if (!first) {
        o->push_back(' ');
        o->append(std::to_string(ts_ns));
        o->push_back('\n');
      } else {
        // no fields: drop the partial line
        size_t p = o->rfind("gpu_ext,");
        if (p != std::string::npos) o->resize(p);
      }
    }
  }
  if (!in.pod_rows) return;
  if (schema == 2018) {
    // The earlier pod_gpu layout still shown in the reference's img/influxdb.png (2018-08-06):
    // columns containerid, gid, gpu, host, namespace, node, pid, pod, procressname, used_gpu (MiB).
    // Idle allocation rows did not exist yet in that version, so they are not emitted here.
    for (const auto& p : *in.pod_rows) {
      if (p.idle) continue;
      const std::string gid = p.dev < static_cast<int>(n) ? st[p.dev].gpu_id : "-";
      o->append("pod_gpu,host=");
      escape_influx_tag(in.host, o);
      o->append(",namespace=");
      escape_influx_tag(p.pod_namespace, o);
      o->append(",gpu=");
      escape_influx_tag(gid, o);
      o->append(",containerid=");
      escape_influx_tag(p.containerid, o);
      o->append(" gid=");
      o->append(gid == "-" ? "-1" : gid);
      o->append(",node=\"");
      escape_influx_field_str(in.host, o);
      o->append("\",pid=\"");
      escape_influx_field_str(p.pid, o);
      o->append("\",pod=\"");
      escape_influx_field_str(p.pod_name, o);
      o->append("\",procressname=\"");
      escape_influx_field_str(p.procname, o);
      o->append("\",used_gpu=");
      append_double(std::floor(p.used_memory_bytes / kMiB), o);
      o->push_back(' ');
      o->append(std::to_string(ts_ns));
      o->push_back('\n');
    }
    return;
  }
  for (const auto& p : *in.pod_rows) {
    const std::string gid = p.dev < static_cast<int>(n) ? st[p.dev].gpu_id : "-";
    // pod_gpu,host,namespace,gpu_id,containerid,pid_t,gpu_util_t,user_name_t  (gpu.py:207-208)
    o->append("pod_gpu,host=");
    escape_influx_tag(in.host, o);
    o->append(",namespace=");
    escape_influx_tag(p.pod_namespace, o);
    o->append(",gpu_id=");
    escape_influx_tag(gid, o);
    o->append(",containerid=");
    escape_influx_tag(p.containerid, o);
    o->append(",pid_t=");
    escape_influx_tag(p.pid, o);
    o->append(",gpu_util_t=");
    std::string gu;
    append_double(p.idle ? 0.0 : p.gpu_util, &gu);
    escape_influx_tag(gu, o);
    o->append(",user_name_t=");
    escape_influx_tag(p.user_name, o);
    // fields (gpu.py:209-216)
    o->append(" procressname=\"");
    escape_influx_field_str(p.procname, o);
    o->append("\",podname=\"");
    escape_influx_field_str(p.pod_name, o);
    o->append("\",pid=\"");
    escape_influx_field_str(p.pid, o);
    o->append("\",gpu_id_v=\"");
    escape_influx_field_str(gid, o);
    o->append("\",node=\"");
    escape_influx_field_str(in.host, o);
    o->append("\",user_name=\"");
    escape_influx_field_str(p.user_name, o);
    o->append("\",gpu_util=");
    append_double(p.idle ? 0.0 : p.gpu_util, o);
    o->append(",used_memory=");
    append_double(std::floor(p.used_memory_bytes / kMiB), o);
    if (extended && !p.idle) {  // per-process fields the reference could not measure (Q4)
      auto extra = [&](const char* k, double x) {
        if (!has(x)) return;
        o->push_back(',');
        o->append(k).push_back('=');
        append_double(x, o);
      };
      extra("proc_gfx_util", p.proc_gfx_util);
      extra("cu_occupancy", p.cu_occupancy);
      extra("mfma_util", p.mfma_util);
    }
    o->push_back(' ');
    o->append(std::to_string(ts_ns));
    o->push_back('\n');
  }
}

}  // namespace gpumon
