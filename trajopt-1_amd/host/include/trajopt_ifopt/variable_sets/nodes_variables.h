// trajopt_ifopt's variable sets (variable_sets/{var,node,nodes_variables}.h):
// a trajectory is a list of Nodes, each holding named Vars (one joint position
// vector per node here); NodesVariables flattens them into the optimisation
// vector, a Var's getIndex() is its first column there.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "trajopt_ifopt/core/bounds.h"
#include "trajopt_ifopt/core/eigen_types.h"

namespace trajopt_ifopt
{
class NodesVariables;

class Var
{
public:
  Var(std::string name, std::vector<std::string> child_names, VectorXd values, std::vector<Bounds> bounds);
  const std::string& getName() const { return name_; }
  const std::vector<std::string>& getChildNames() const { return child_names_; }
  Index getIndex() const { return index_; }  // first column in the flat variable vector
  Index size() const { return static_cast<Index>(values_.size()); }
  const VectorXd& value() const { return values_; }
  const std::vector<Bounds>& getBounds() const { return bounds_; }

private:
  friend class NodesVariables;
  std::string name_;
  std::vector<std::string> child_names_;
  VectorXd values_;
  std::vector<Bounds> bounds_;
  Index index_ = -1;
};

class Node
{
public:
  explicit Node(std::string name) : name_(std::move(name)) {}
  std::shared_ptr<const Var> addVar(const std::string& name, const std::vector<std::string>& child_names,
                                    const VectorXd& values, const std::vector<Bounds>& bounds);
  const std::string& getName() const { return name_; }
  const std::vector<std::shared_ptr<Var>>& getVars() const { return vars_; }

private:
  std::string name_;
  std::vector<std::shared_ptr<Var>> vars_;
};

class NodesVariables
{
public:
  using Ptr = std::shared_ptr<NodesVariables>;
  NodesVariables(std::string name, std::vector<std::unique_ptr<Node>> nodes);
  const std::string& getName() const { return name_; }
  Index getRows() const { return rows_; }
  VectorXd getValues() const;
  void setVariables(const VectorXd& x);
  std::vector<Bounds> getBounds() const;
  // changes whenever setVariables changes a value (TrajOptQPProblem skips term updates otherwise)
  std::size_t getHash() const { return hash_; }

private:
  std::string name_;
  std::vector<std::unique_ptr<Node>> nodes_;
  std::vector<std::shared_ptr<Var>> vars_;
  Index rows_ = 0;
  std::size_t hash_ = 0;
};
using Variables = NodesVariables;
}  // namespace trajopt_ifopt
