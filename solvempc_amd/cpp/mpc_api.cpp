// solvempc_amd/cpp/mpc_api.cpp — ModelPredictiveControlAPI on MI355X (see mpc_api.hpp).
#include "mpc_api.hpp"

#include <algorithm>
#include <cfloat>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

using mpcq::Matrix;

ModelPredictiveControlAPI::ModelPredictiveControlAPI(bool verbose_, const std::string &config, int N, int device)
    : solver(device), horizon(N), device_(device)
{
    std::cout << "[MPC API]\tMPC API object created." << std::endl;
    verbose = verbose_;
    solverFlag = true;
    std::ifstream file(config);  // CWD-relative by default, like the reference (:12)
    if (!file) throw json_lite::error("parse_error: cannot open " + config);
    std::stringstream ss;
    ss << file.rdbuf();
    cfg = json_lite::parse(ss.str());
    K = from_json(cfg["K"], 1, N_S);
    xref = cfg["xref"].get_double();
    X = Matrix::Zero(N_S, 1);
    U = Matrix::Zero(N_O, N_O);
    t0 = dt = 0.0;

    setSystemVars();
    setCosts();
    setLiftedCosts();
    setTransformations();
    setLL();
    setH();
    setLu();
    setFVars();
    setLinearConstraints();
    setUpperBound();
    updateRef(xref);
    setF();

    lb = Matrix(2 * horizon, 1, -DBL_MAX);  // :42
    ub = Matrix(2 * horizon, 1);            // :43  W0 + Sbar X + Ku U
    for (int i = 0; i < 2 * horizon; i++) {
        double s = 0.0;
        for (int c = 0; c < N_S; c++) s += Sbar(i, c) * X(c);
        ub(i) = W0(i) + s + Ku(i) * U(0);
    }
    std::cout << "[MPC API]\tAll QP matrices built successfully." << std::endl;

    n_variables = N_O * horizon;
    n_constraints = 2 * horizon;
    solver.settings()->setVerbosity(verbose);
    solver.settings()->setWarmStart(true);
    solver.data()->setNumberOfVariables(n_variables);
    solver.data()->setNumberOfConstraints(n_constraints);
    if (!solver.data()->setHessianMatrix(H)) { solverFlag = false; return; }
    if (!solver.data()->setGradient(std::vector<double>(f.data(), f.data() + f.size()))) { solverFlag = false; return; }
    if (!solver.data()->setLinearConstraintsMatrix(Gbar)) { solverFlag = false; return; }
    if (!solver.data()->setLowerBound(std::vector<double>(lb.data(), lb.data() + lb.size()))) { solverFlag = false; return; }
    if (!solver.data()->setUpperBound(std::vector<double>(ub.data(), ub.data() + ub.size()))) { solverFlag = false; return; }
    if (!solver.initSolver()) { solverFlag = false; return; }
}

ModelPredictiveControlAPI::~ModelPredictiveControlAPI()
{
    std::printf("[MPC API]\tDestructing MPC API object...\n");
}

void ModelPredictiveControlAPI::setVerbosity(bool v)
{
    verbose = v;
    std::cout << "[MPC API]\tVerbosity set to " << verbose << std::endl;
}

void ModelPredictiveControlAPI::setSystemVars()
{
    Ad = from_json(cfg["Ad"], N_S, N_S);
    Bd = from_json(cfg["Bd"], N_S, N_C);
    Cd = from_json(cfg["Cd"], N_O, N_S);
    Dd = from_json(cfg["Dd"], N_O, N_C);
    if (verbose) std::cout << "[MPC API]\tSystem variables created." << std::endl;
}

void ModelPredictiveControlAPI::setCosts()
{
    Q = from_json(cfg["Q"], N_O, N_O);
    R = from_json(cfg["R"], N_O, N_O);
    RD = from_json(cfg["RD"], N_O, N_O);
    if (verbose) std::cout << "[MPC API]\tSet Q, R, and RD matrices created." << std::endl;
}

void ModelPredictiveControlAPI::setLiftedCosts()
{
    Qbar = blkdiag(Q, horizon);
    Rbar = blkdiag(R, horizon);
    RbarD = blkdiag(RD, horizon);
    if (verbose) std::cout << "[MPC API]\tLifted weight matrices created." << std::endl;
}

// The condensed operators come from the device kernel (mpcq_condense), built once here and
// handed out by the individual set* builders below.
void ModelPredictiveControlAPI::condense_on_device()
{
    const int N = horizon;
    std::vector<double> P(N * N), A(2 * N * N), fx(N * N_S), fu(N), fr(N * N), sbar(2 * N * N_S), ku(2 * N), w0(2 * N);
    const std::vector<double> ad = Ad.row_major(), bd = Bd.row_major(), cd = Cd.row_major(), k = K.row_major();
    const double q = Q(0, 0), r = R(0, 0), rd = RD(0, 0);
    if (mpcq_condense(device_, 1, N_S, N, 10, ad.data(), bd.data(), cd.data(), k.data(), &q, &r, &rd, P.data(),
                      A.data(), fx.data(), fu.data(), fr.data(), sbar.data(), ku.data(), w0.data()) != MPCQ_OK)
        throw std::runtime_error(std::string("[MPC API]\tcondensing failed: ") + mpcq_last_error());
    H = Matrix::from_row_major(N, N, P.data());
    Gbar = Matrix::from_row_major(2 * N, N, A.data());
    Fx = Matrix::from_row_major(N, N_S, fx.data());
    Fu = Matrix::from_row_major(N, 1, fu.data());
    Fr = Matrix::from_row_major(N, N, fr.data());
    Sbar = Matrix::from_row_major(2 * N, N_S, sbar.data());
    Ku = Matrix::from_row_major(2 * N, 1, ku.data());
    W0 = Matrix::from_row_major(2 * N, 1, w0.data());
    S = Matrix(N, N_S);
    for (int i = 0; i < N; i++)
        for (int c = 0; c < N_S; c++) S(i, c) = Sbar(i, c);
    condensed_ = true;
}

void ModelPredictiveControlAPI::setTransformations()
{
    if (!condensed_) condense_on_device();
    if (verbose) std::cout << "[MPC API]\tTransformation matrices created" << std::endl;
}

void ModelPredictiveControlAPI::setH()
{
    if (!condensed_) condense_on_device();
    if (verbose) std::cout << "[MPC API]\tHessian H created." << std::endl;
}

void ModelPredictiveControlAPI::setLu()
{
    Lu = Matrix(horizon, 1);  // (mpcWindow - i + 2), unused by the QP (:274-279)
    for (int i = 0; i < horizon; i++) Lu(i) = horizon - i + 2;
}

void ModelPredictiveControlAPI::setLL()
{
    LL = Matrix(horizon, horizon);
    for (int i = 0; i < horizon; i++)
        for (int j = 0; j <= i; j++) LL(i, j) = 1.0;
}

void ModelPredictiveControlAPI::setFVars()
{
    if (!condensed_) condense_on_device();
    if (verbose) std::cout << "[MPC API]\tComponents of F created." << std::endl;
}

void ModelPredictiveControlAPI::setLinearConstraints()
{
    if (!condensed_) condense_on_device();
    if (verbose) std::cout << "[MPC API]\tLinear constraints matrix created." << std::endl;
}

void ModelPredictiveControlAPI::setUpperBound()
{
    // Ku = [-K0 1; K0 1], W0 = 255 1 (:364-368) — constants, already on the condensed result
    if (!condensed_) condense_on_device();
}

void ModelPredictiveControlAPI::setF()
{
    // f = Fx X + Fu U + Fr ref'  (:374)
    f = Matrix(horizon, 1);
    for (int i = 0; i < horizon; i++) {
        double a = 0.0, c = 0.0;
        for (int t = 0; t < N_S; t++) a += Fx(i, t) * X(t);
        const double b = Fu(i) * U(0);
        for (int t = 0; t < horizon; t++) c += Fr(i, t) * ref(t);
        f(i) = a + b + c;
    }
}

void ModelPredictiveControlAPI::updateRef(double pos_ref)
{
    ref = Matrix(1, horizon, pos_ref);
    if (verbose) std::cout << "[MPC API]\tref: " << pos_ref << std::endl;
}

bool ModelPredictiveControlAPI::controllerStep()
{
    t0 += dt;
    updateRef(xref);
    setF();
    setUpperBound();
    if (!solver.updateGradient(std::vector<double>(f.data(), f.data() + f.size()))) return false;
    std::vector<double> u(2 * horizon);
    for (int i = 0; i < 2 * horizon; i++) {
        double s = 0.0;
        for (int c = 0; c < N_S; c++) s += Sbar(i, c) * X(c);
        u[i] = W0(i) + s + Ku(i) * U(0);
    }
    if (!solver.updateUpperBound(u)) return false;
    if (!solver.solve()) return false;
    U(0) += solver.getSolution()[0];  // receding horizon (:105)
    return true;
}

Matrix ModelPredictiveControlAPI::blkdiag(const Matrix &a, int count)
{
    Matrix b(a.rows() * count, a.cols() * count);
    for (int i = 0; i < count; i++)
        for (int r = 0; r < a.rows(); r++)
            for (int c = 0; c < a.cols(); c++) b(i * a.rows() + r, i * a.cols() + c) = a(r, c);
    return b;
}

// from_json shape rules of the reference (:418-489): scalar, row/column vector or matrix.
Matrix ModelPredictiveControlAPI::from_json(const json_lite::Value &j, int rows, int cols)
{
    std::vector<const json_lite::Value *> flat;
    json_lite::Value arr;
    if (j.is_array()) {
        if (j.empty()) return Matrix(rows, cols);
        arr = j;
    } else if (j.is_number()) {
        arr.kind = json_lite::Value::Array;
        arr.arr.push_back(j);
    } else {
        throw json_lite::error("type_error: expected a number or an array");
    }
    std::vector<std::vector<double>> aoa;
    if (arr.arr.front().is_array()) {
        for (const auto &row : arr.arr) {
            std::vector<double> r;
            if (!row.is_array()) throw json_lite::error("type_error: mixed rows");
            for (const auto &v : row.arr) r.push_back(v.get_double());
            aoa.push_back(r);
        }
    } else if (rows == 1) {
        std::vector<double> r;
        for (const auto &v : arr.arr) r.push_back(v.get_double());
        aoa.push_back(r);
    } else if (cols == 1) {
        for (const auto &v : arr.arr) aoa.push_back({v.get_double()});
    } else {
        std::cerr << "Expected a matrix, received a vector." << std::endl;
        throw json_lite::error("type_error: expected a matrix");
    }
    const int pr = (int)aoa.size(), pc = (int)aoa.front().size();
    if ((rows >= 0 && pr != rows) || (cols >= 0 && pc != cols)) {
        std::cerr << "Expected matrix of size " << rows << "x" << cols << ", received matrix of size " << pr << "x" << pc
                  << "." << std::endl;
        throw json_lite::error("type_error: size mismatch");
    }
    Matrix m(pr, pc);
    for (int r = 0; r < pr; r++) {
        if ((int)aoa[r].size() != pc) {
            std::cerr << "Unconsistent matrix size: some rows have different number of columns." << std::endl;
            throw json_lite::error("type_error: ragged rows");
        }
        for (int c = 0; c < pc; c++) m(r, c) = aoa[r][c];
    }
    return m;
}

char *getCmdOption(char **begin, char **end, const std::string &option)
{
    char **itr = std::find(begin, end, option);
    if (itr != end && ++itr != end) return *itr;
    return nullptr;
}

bool cmdOptionExists(char **begin, char **end, const std::string &option)
{
    return std::find(begin, end, option) != end;
}
