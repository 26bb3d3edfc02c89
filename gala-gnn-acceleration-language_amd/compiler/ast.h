// ast.h — syntax tree of a GALA DSL program.
//
// The language is the one tests/GALA-DSL/** programs are written in (lexicon
// src/frontend/frontend.l:23-138, grammar src/frontend/frontend.y:70-437).  The reference
// builds it with bison/flex, which this image lacks; this is a hand-written
// recursive-descent parser over a general expression grammar, so the shapes the
// reference's grammar hard-codes (e.g. `aggrFn=aggrFn.sample(20).dynamic();`) are just
// member-call chains here and are given meaning in lower.cpp.
#pragma once

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace galac {

struct SrcLoc {
    int line = 0, col = 0;
};

class DslError : public std::runtime_error {
  public:
    DslError(const SrcLoc &at, const std::string &msg)
        : std::runtime_error("line " + std::to_string(at.line) + ":" + std::to_string(at.col) +
                             ": " + msg),
          loc(at) {}
    SrcLoc loc;
};

struct Expr;
using ExprP = std::shared_ptr<Expr>;

struct Expr {
    enum Kind { Ident, Number, String, Bool, Null, Member, Call, Binary, Neg };
    Kind kind;
    SrcLoc at;
    std::string name;               // Ident / Member field / Binary operator ("+-*/")
    double num = 0;                 // Number
    bool is_int = false;            // Number written without '.' / exponent
    bool bval = false;              // Bool
    ExprP obj;                      // Member object, Call callee, Neg operand
    ExprP lhs, rhs;                 // Binary
    std::vector<ExprP> args;        // Call arguments
    std::vector<std::string> kw;    // Call keyword per argument ("" = positional)

    // Dotted path of an Ident/Member chain ("dsl.fn.mul_sum"), "" if not a pure path.
    std::string path() const;
};

struct Stmt;
using StmtP = std::shared_ptr<Stmt>;

struct Stmt {
    enum Kind { Assign, Eval, Block };
    Kind kind;
    SrcLoc at;
    ExprP target;                   // Assign: Ident or Member path
    ExprP value;                    // Assign / Eval
    // Block: `name = layer(params) { body }` or `name = model(params) { body }`
    std::string block_kind, block_name;
    std::vector<std::string> params;
    std::vector<StmtP> body;
};

struct Program {
    std::string source_name;
    std::vector<StmtP> stmts;
};

Program parse_program(const std::string &text, const std::string &source_name);
Program parse_file(const std::string &path);

}  // namespace galac
