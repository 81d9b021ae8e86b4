// solvempc_amd/cpp/mpc_api.hpp — drop-in C++ surface of the reference's ModelPredictiveControlAPI
// (include/ModelPredictiveControlAPI.h:47-243 of LukeSchmitt96/solveMPC), running its QP on MI355X.
//
// Kept: the constructor ModelPredictiveControlAPI(bool verbose) reading ./config/MPC_API.json,
// setVerbosity, the set* builders, updateRef, setF, controllerStep() -> bool, the public members
// (X, U, dt, t0, verbose, solverFlag, n_variables, n_constraints, cfg, the QP operators) and the
// "[MPC API]" log tags.  Changed: matrices are mpcq::Matrix (no Eigen), the horizon is a constructor
// argument defaulting to the reference's mpcWindow = 15 (ModelPredictiveControlAPI.h:26), the QP
// operators are built by the device condensing kernel (mpcq_condense) and the solver is
// mpcq::Solver (osqp-eigen surface over the C ABI).
#pragma once

#include <stdexcept>
#include <string>

#include "json_lite.hpp"
#include "mpcq_solver.hpp"

constexpr int mpcWindow = 15;  // default horizon (reference: compile-time constant)
constexpr int N_S = 4;         // states
constexpr int N_C = 1;         // controls
constexpr int N_O = 1;         // outputs

// A device-side build step of the constructor failed (no usable device): the constructor reports it and
// leaves solverFlag false, the reference's failure exit.
struct DeviceError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class ModelPredictiveControlAPI {
public:
    explicit ModelPredictiveControlAPI(bool verbose_, const std::string &config = "./config/MPC_API.json",
                                       int horizon = mpcWindow, int device = 0);
    ~ModelPredictiveControlAPI();

    void setVerbosity(bool);
    void setSystemVars();
    void setCosts();
    void setLiftedCosts();
    void setTransformations();
    void setH();
    void setFVars();
    void setLinearConstraints();
    void setF();
    void setUpperBound();
    void updateRef(double pos_ref);
    void setLL();
    void setLu();
    bool controllerStep();

    mpcq::Solver solver;
    bool solverFlag = true;

    // system matrices (ModelPredictiveControlAPI.h:148-200)
    mpcq::Matrix Ad, Bd, Cd, Dd;
    mpcq::Matrix Q, R, RD, Qbar, Rbar, RbarD;
    mpcq::Matrix S, Sbar, W0, Gbar, LL, Lu;
    mutable mpcq::Matrix Sx, Su, Su1;  // printed by the -v dump only (the device kernel forms the QP)
    mpcq::Matrix X, U, ref, K, Ku;
    double xref = 0.0;
    mpcq::Matrix H, Fu, Fr, Fx, f, lb, ub;
    double t0 = 0.0, dt = 0.0;
    int n_variables = 0, n_constraints = 0;
    int horizon;
    bool verbose = false;
    json_lite::Value cfg;

    static mpcq::Matrix from_json(const json_lite::Value &jsonObject, int rows, int cols);
    static mpcq::Matrix blkdiag(const mpcq::Matrix &a, int count);

private:
    void condense_on_device();
    void transformations_for_dump(mpcq::Matrix &CAB, mpcq::Matrix &CAiB, mpcq::Matrix &CAB_full, mpcq::Matrix &Su_full,
                                  mpcq::Matrix &Su_full1) const;
    bool condensed_ = false;
    int device_;
};

// solver.h surface (include/solver.h:22,27; src/solver.cpp:83-97)
char *getCmdOption(char **begin, char **end, const std::string &option);
bool cmdOptionExists(char **begin, char **end, const std::string &option);
