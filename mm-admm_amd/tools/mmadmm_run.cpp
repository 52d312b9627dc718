// mmadmm_run -- experiment driver with the reference's command line, config files and outputs
// (SURVEY.md §8f row 1): `mmadmm_run <testName> [method] [numThreads]` reads
// Experiments/InputFiles/<testName>.json, builds the mesh, runs the time loop and writes
// Experiments/Results/<testName>/{points.txt, triangles.txt, Ih<method>.txt, IhPara<threads>.txt}
// exactly as main.cpp's main/runAlgo (main.cpp:132-255, 633-907) do, on the MI355X engine through
// the C-ABI of include/mmadmm.h.
//
// Supported: TestType FromFile, SquareGrid, LevelSet (2D circlePhi, 3D spherePhi), Shoulder (glibc
// rand after srand(69) as main.cpp:785, Eigen 3.4 Random semantics); Method 0 (ADMM), 1 (explicit
// Euler) and 2 (backward Euler: Newton + ILU(0) CG-STAB).  Extra options: --root DIR (instead of the current directory), --device N,
// --dry-run (parse and build the mesh on the host only; no GPU).
#include <sys/stat.h>
#include <time.h>

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "mmadmm.h"

namespace {

// ---- a small JSON reader for the reference's flat config objects -------------------------------
struct JVal {
  enum Kind { NUM, STR, BOOL, NUL, OTHER } kind = NUL;
  double num = 0;
  std::string str;
  bool b = false;
};

class JsonFlat {
 public:
  explicit JsonFlat(const std::string& text) : s_(text) {}
  std::map<std::string, JVal> parse() {
    std::map<std::string, JVal> out;
    ws();
    expect('{');
    ws();
    if (peek() == '}') return out;
    while (true) {
      ws();
      const std::string key = str();
      ws();
      expect(':');
      ws();
      out[key] = value();
      ws();
      if (peek() == ',') {
        ++p_;
        continue;
      }
      expect('}');
      break;
    }
    return out;
  }

 private:
  char peek() const { return p_ < s_.size() ? s_[p_] : '\0'; }
  void ws() {
    while (p_ < s_.size() && std::isspace((unsigned char)s_[p_])) ++p_;
  }
  void expect(char c) {
    if (peek() != c) throw std::runtime_error(std::string("config: expected '") + c + "' at offset " + std::to_string(p_));
    ++p_;
  }
  std::string str() {
    expect('"');
    std::string r;
    while (p_ < s_.size() && s_[p_] != '"') {
      if (s_[p_] == '\\' && p_ + 1 < s_.size()) ++p_;
      r += s_[p_++];
    }
    expect('"');
    return r;
  }
  JVal value() {
    JVal v;
    const char c = peek();
    if (c == '"') {
      v.kind = JVal::STR;
      v.str = str();
    } else if (s_.compare(p_, 4, "true") == 0) {
      v.kind = JVal::BOOL;
      v.b = true;
      p_ += 4;
    } else if (s_.compare(p_, 5, "false") == 0) {
      v.kind = JVal::BOOL;
      p_ += 5;
    } else if (s_.compare(p_, 4, "null") == 0) {
      p_ += 4;
    } else if (c == '{' || c == '[') {  // nested values are skipped (the reference has none)
      v.kind = JVal::OTHER;
      int depth = 0;
      do {
        if (s_[p_] == '{' || s_[p_] == '[') ++depth;
        if (s_[p_] == '}' || s_[p_] == ']') --depth;
        ++p_;
      } while (depth > 0 && p_ < s_.size());
    } else {
      v.kind = JVal::NUM;
      size_t used = 0;
      v.num = std::stod(s_.substr(p_), &used);
      p_ += used;
    }
    return v;
  }
  std::string s_;
  size_t p_ = 0;
};

struct Config {
  std::map<std::string, JVal> kv;
  bool has(const std::string& k) const { return kv.count(k) != 0; }
  double num(const std::string& k) const {
    auto it = kv.find(k);
    if (it == kv.end()) throw std::runtime_error("config: missing key " + k);
    if (it->second.kind == JVal::BOOL) return it->second.b ? 1.0 : 0.0;
    if (it->second.kind != JVal::NUM) throw std::runtime_error("config: key " + k + " is not a number");
    return it->second.num;
  }
  int integer(const std::string& k) const { return (int)num(k); }  // json int conversion
  std::string str(const std::string& k) const {
    auto it = kv.find(k);
    if (it == kv.end() || it->second.kind != JVal::STR) throw std::runtime_error("config: missing string " + k);
    return it->second.str;
  }
};

void check(int rc, const char* what) {
  if (rc != MMADMM_OK) {
    std::cerr << what << ": " << mmadmm_last_error() << std::endl;
    std::exit(1);
  }
}

// outputVecToFile (main.cpp:132-140): "t, I" rows with the default ostream format
void outputVecToFile(const std::string& fileName, const std::vector<double>& t, const std::vector<double>& v) {
  std::ofstream out(fileName);
  for (size_t i = 0; i < t.size(); i++) out << t.at(i) << ", " << v.at(i) << std::endl;
}

void mkdirs(const std::string& path) {
  std::string cur;
  std::stringstream ss(path);
  std::string part;
  if (!path.empty() && path[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    mkdir(cur.c_str(), 0755);
  }
}

double now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec / 1e9;
}

}  // namespace

int main(int argc, char** argv) {
  srand(69);  // main.cpp:785 (the Shoulder experiment's random perturbation)
  std::vector<std::string> pos;
  std::string root = ".";
  int device = 0;
  bool dry = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--root" && i + 1 < argc) root = argv[++i];
    else if (a == "--device" && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (a == "--dry-run") dry = true;
    else pos.push_back(a);
  }
  if (pos.empty()) {
    std::cerr << "usage: mmadmm_run <testName> [method] [numThreads] [--root DIR] [--device N] [--dry-run]"
              << std::endl;
    return 2;
  }
  const std::string testName = pos[0];
  const int methodType = pos.size() >= 2 ? std::atoi(pos[1].c_str()) : 0;
  const int numThreads = pos.size() >= 3 ? std::atoi(pos[2].c_str()) : 1;

  Config cfg;
  try {
    const std::string fname = root + "/Experiments/InputFiles/" + testName + ".json";
    std::ifstream in(fname);
    if (!in) throw std::runtime_error("cannot read " + fname);
    std::stringstream buf;
    buf << in.rdbuf();
    cfg.kv = JsonFlat(buf.str()).parse();
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }

  try {
    const std::string testType = cfg.str("TestType");
    const int D = cfg.integer("Dim");
    const int monType = cfg.integer("MonType");
    const int boundaryType = cfg.integer("BoundaryType");
    const int btype = boundaryType == 0 ? MMADMM_BOUNDARY_FREE : MMADMM_BOUNDARY_FIXED;
    const bool compMesh = cfg.num("CompMesh") != 0;
    const bool gradUse = cfg.num("GradUse") != 0;
    const int admmIter = cfg.integer("AdmmIter");
    const double dtTol = cfg.num("DtTol");
    const int nSteps = cfg.integer("nSteps");
    bool shoulder = false;
    const double dt = cfg.num("dt"), tau = cfg.num("tau"), rho = cfg.num("rho");
    std::cout << "testName " << testName << " TestType " << testType << " Dim " << D << " Method " << methodType
              << std::endl;
    if (methodType < 0 || methodType > 2) {
      std::cerr << "unknown Method " << methodType << std::endl;
      return 2;
    }

    mmadmm_mesh mesh = nullptr;
    if (testType == "FromFile") {  // setUpFileExperiment (main.cpp:736-782)
      auto path = [&](const std::string& k) {
        std::string f = cfg.str(k);
        return (f.rfind("./", 0) == 0 ? root + "/" + f.substr(2) : (f[0] == '/' ? f : root + "/" + f));
      };
      // some of the reference's input meshes were never committed (its .MISSING_LARGE_BLOBS):
      // such a config is reported as unavailable, not as a failure of the run
      for (const char* k : {"TrianglesFile", "PntsFile", "MaskFile"}) {
        struct stat sb;
        if (stat(path(k).c_str(), &sb) != 0) {
          std::cerr << "FromFile mesh " << path(k) << " is not available (" << k << " missing)" << std::endl;
          return 2;
        }
      }
      check(mmadmm_mesh_read(D, path("TrianglesFile").c_str(), path("PntsFile").c_str(), path("MaskFile").c_str(),
                             &mesh),
            "readTriangles");
    } else if (testType == "SquareGrid") {  // setUpBoxExperiment (main.cpp:633-734)
      const int nx = cfg.integer("nx"), ny = cfg.integer("ny"), nz = D == 3 ? cfg.integer("nz") : 0;
      const double za = D == 3 ? cfg.num("za") : 0.0, zb = D == 3 ? cfg.num("zb") : 0.0;
      check(mmadmm_mesh_rect(D, nx, ny, nz, cfg.num("xa"), cfg.num("xb"), cfg.num("ya"), cfg.num("yb"), za, zb,
                             btype, &mesh),
            "generateUniformRectMesh");
    } else if (testType == "Shoulder") {  // setUpShoulderExperiment (main.cpp:403-630)
      const int nx = cfg.integer("nx"), ny = cfg.integer("ny"), nz = D == 3 ? cfg.integer("nz") : 0;
      const double za = D == 3 ? cfg.num("za") : 0.0, zb = D == 3 ? cfg.num("zb") : 0.0;
      check(mmadmm_mesh_shoulder(D, nx, ny, nz, cfg.num("xa"), cfg.num("xb"), cfg.num("ya"), cfg.num("yb"), za, zb,
                                 btype, &mesh),
            "setUpShoulderExperiment");
      shoulder = true;
    } else if (testType == "LevelSet" && D == 2) {  // setUpLevelSetExperiment (main.cpp:258-402)
      check(mmadmm_mesh_levelset2d(cfg.integer("nx"), cfg.integer("ny"), cfg.num("xa"), cfg.num("xb"), cfg.num("ya"),
                                   cfg.num("yb"), btype, 0, &mesh),
            "meshFromLevelSetFun");
    } else if (testType == "LevelSet" && D == 3) {  // the same, 3D (spherePhi, main.cpp:363-371)
      // the reference's 3D generator loses its result (MeshUtils.h:663-666); this one returns it,
      // with the mask remapped to the new node numbering
      check(mmadmm_mesh_levelset3d(cfg.integer("nx"), cfg.integer("ny"), cfg.integer("nz"), cfg.num("xa"),
                                   cfg.num("xb"), cfg.num("ya"), cfg.num("yb"), cfg.num("za"), cfg.num("zb"), btype,
                                   1, &mesh),
            "meshFromLevelSetFun");
    } else {
      std::cerr << "TestType " << testType << " (Dim " << D << ") is not available in this build" << std::endl;
      return 2;
    }
    int dim = 0, nP = 0, nF = 0, maskLen = 0;
    check(mmadmm_mesh_sizes(mesh, &dim, &nP, &nF, &maskLen), "mesh sizes");
    std::vector<double> Xp((size_t)nP * D);
    std::vector<int32_t> F((size_t)nF * (D + 1)), mask(maskLen);
    check(mmadmm_mesh_copy(mesh, Xp.data(), F.data(), mask.data()), "mesh copy");
    std::vector<double> Xc(Xp);  // CompMesh reference: the initial Vp, or Shoulder's unmoved Vc
    if (shoulder) check(mmadmm_mesh_reference_points(mesh, Xc.data()), "mesh reference points");
    mmadmm_mesh_free(mesh);
    std::cout << "size of Vp " << nP << ", " << D << std::endl;
    std::cout << "size of F " << nF << ", " << D + 1 << std::endl;
    std::cout << "size of mask " << maskLen << std::endl;
    if (dry) return 0;

    mmadmm_monitor_fn fn = nullptr;
    void* user = nullptr;
    check(mmadmm_builtin_monitor(D, monType, &fn, &user), "monitor");
    mmadmm_params p{};
    p.dt = dt;
    p.tau = tau;
    p.rho = rho;
    p.grad_use = gradUse ? 1 : 0;
    p.device = device;
    p.rank = 0;
    p.nranks = 1;
    mmadmm_handle h = nullptr;
    // CompMesh: Vc is a copy of the initial Vp (main.cpp:727, 778) or Shoulder's unmoved mesh (main.cpp:479-491)
    check(mmadmm_create(D, nP, Xp.data(), compMesh ? Xc.data() : nullptr, nF, F.data(), mask.data(), &p, fn, user,
                        &h),
          "Mesh/MeshIntegrator");

    // runAlgo (main.cpp:142-255)
    std::vector<double> Ivals, tVals;
    double E = 0;
    check(mmadmm_energy(h, &E), "getEnergy");
    Ivals.push_back(E);
    tVals.push_back(0);
    const double start = now();
    double Ih = 0, Ihprev = INFINITY;
    int i;
    for (i = 0; i < nSteps; i++) {
      if (methodType == 0) {
        int it = 0;
        check(mmadmm_step(h, admmIter, 1e-3, &Ih, &it), "step");
      } else if (methodType == 1) {
        check(mmadmm_euler_step(h, &Ih), "eulerStep");
      } else {
        int newton = 0;
        check(mmadmm_backward_euler_step(h, dt, 1e-3, &Ih, &newton), "backwardsEulerStep");
        std::cout << "Newton in " << newton << " iters" << std::endl;
      }
      Ivals.push_back(Ih);
      tVals.push_back(now() - start);
      const double dIdt = (Ih - Ihprev) / dt;
      if (i != 0 && (std::abs(dIdt) < dtTol)) {
        std::cout << "converged" << std::endl;
        break;
      }
      Ihprev = Ih;
    }
    const double elapsed = now() - start;
    std::cout << "Took " << elapsed << " seconds" << std::endl;
    std::cout << "Took " << i << " iters" << std::endl;
    std::cout << "Number of simplices = " << nF << std::endl;
    std::cout << "Number of points = " << nP << std::endl;
    check(mmadmm_done(h), "done");

    const std::string outDir = root + "/Experiments/Results/" + testName;
    mkdirs(outDir);
    std::vector<double> pts((size_t)nP * D);
    check(mmadmm_get(h, "points", pts.data()), "points");
    check(mmadmm_get_simplices(h, F.data()), "simplices");
    check(mmadmm_write_points((outDir + "/points.txt").c_str(), D, nP, pts.data()), "outputPoints");
    check(mmadmm_write_simplices((outDir + "/triangles.txt").c_str(), D, nF, F.data()), "outputSimplices");
    outputVecToFile(outDir + "/IhPara" + std::to_string(numThreads) + ".txt", tVals, Ivals);
    if (numThreads == 1) outputVecToFile(outDir + "/Ih" + std::to_string(methodType) + ".txt", tVals, Ivals);
    mmadmm_destroy(h);
  } catch (const std::exception& e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }
  return 0;
}
