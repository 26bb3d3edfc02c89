// parser.cpp — lexer + recursive-descent parser for the GALA DSL (see ast.h).
//
//   program   := stmt*
//   stmt      := IDENT '=' ('layer'|'model') '(' params ')' '{' stmt* '}'
//              | expr ('=' expr)? ';'
//   expr      := term (('+'|'-') term)*
//   term      := unary (('*'|'/') unary)*
//   unary     := '-' unary | postfix
//   postfix   := primary ('.' IDENT | '(' args ')')*
//   primary   := IDENT | NUMBER | STRING | 'true' | 'false' | 'null' | '(' expr ')'
//   args      := (arg (',' arg)*)?        arg := (IDENT '=')? expr
//
// Comments run from `//` or `#` to the end of the line (frontend.l:23-25 skips `//`
// comments; the shipped programs also use a `# schedule` line).
#include <cctype>
#include <fstream>
#include <sstream>

#include "ast.h"

namespace galac {

std::string Expr::path() const {
    if (kind == Ident) return name;
    if (kind == Member && obj) {
        const std::string p = obj->path();
        return p.empty() ? std::string() : p + "." + name;
    }
    return {};
}

namespace {

struct Token {
    enum Kind { Ident, Number, String, Punct, End };
    Kind kind;
    std::string text;
    SrcLoc at;
};

std::vector<Token> lex(const std::string &s) {
    std::vector<Token> out;
    int line = 1, col = 1;
    size_t i = 0;
    auto adv = [&](size_t n) {
        for (size_t k = 0; k < n; ++k, ++i) {
            if (s[i] == '\n') {
                ++line;
                col = 1;
            } else {
                ++col;
            }
        }
    };
    while (i < s.size()) {
        const char c = s[i];
        if (std::isspace((unsigned char)c)) {
            adv(1);
            continue;
        }
        if (c == '#' || (c == '/' && i + 1 < s.size() && s[i + 1] == '/')) {
            while (i < s.size() && s[i] != '\n') adv(1);
            continue;
        }
        const SrcLoc at{line, col};
        if (std::isalpha((unsigned char)c) || c == '_') {
            size_t j = i;
            while (j < s.size() && (std::isalnum((unsigned char)s[j]) || s[j] == '_')) ++j;
            out.push_back({Token::Ident, s.substr(i, j - i), at});
            adv(j - i);
        } else if (std::isdigit((unsigned char)c) ||
                   (c == '.' && i + 1 < s.size() && std::isdigit((unsigned char)s[i + 1]))) {
            size_t j = i;
            while (j < s.size() && std::isdigit((unsigned char)s[j])) ++j;
            if (j < s.size() && s[j] == '.') {
                ++j;
                while (j < s.size() && std::isdigit((unsigned char)s[j])) ++j;
            }
            if (j < s.size() && (s[j] == 'e' || s[j] == 'E')) {
                size_t k = j + 1;
                if (k < s.size() && (s[k] == '+' || s[k] == '-')) ++k;
                if (k < s.size() && std::isdigit((unsigned char)s[k])) {
                    j = k;
                    while (j < s.size() && std::isdigit((unsigned char)s[j])) ++j;
                }
            }
            out.push_back({Token::Number, s.substr(i, j - i), at});
            adv(j - i);
        } else if (c == '"') {
            size_t j = i + 1;
            while (j < s.size() && s[j] != '"' && s[j] != '\n') ++j;
            if (j >= s.size() || s[j] != '"') throw DslError(at, "unterminated string");
            out.push_back({Token::String, s.substr(i + 1, j - i - 1), at});
            adv(j + 1 - i);
        } else if (std::string("=(){},;.+-*/").find(c) != std::string::npos) {
            out.push_back({Token::Punct, std::string(1, c), at});
            adv(1);
        } else {
            throw DslError(at, std::string("unexpected character '") + c + "'");
        }
    }
    out.push_back({Token::End, "", {line, col}});
    return out;
}

class Parser {
  public:
    explicit Parser(std::vector<Token> t) : toks_(std::move(t)) {}

    std::vector<StmtP> statements(bool in_block) {
        std::vector<StmtP> out;
        while (true) {
            if (peek().kind == Token::End) {
                if (in_block) throw DslError(peek().at, "missing '}'");
                return out;
            }
            if (in_block && is_punct("}")) return out;
            out.push_back(statement());
        }
    }

  private:
    std::vector<Token> toks_;
    size_t p_ = 0;

    const Token &peek(size_t k = 0) const { return toks_[std::min(p_ + k, toks_.size() - 1)]; }
    bool is_punct(const char *s, size_t k = 0) const {
        return peek(k).kind == Token::Punct && peek(k).text == s;
    }
    const Token &next() { return toks_[std::min(p_++, toks_.size() - 1)]; }
    void expect(const char *s) {
        if (!is_punct(s)) {
            const Token &t = peek();
            throw DslError(t.at, std::string("expected '") + s + "' but found '" +
                                     (t.kind == Token::End ? "end of file" : t.text) + "'");
        }
        ++p_;
    }
    std::string ident() {
        if (peek().kind != Token::Ident) throw DslError(peek().at, "expected an identifier");
        return next().text;
    }

    StmtP statement() {
        // block definition: IDENT '=' layer|model '(' params ')' '{'
        if (peek().kind == Token::Ident && is_punct("=", 1) && peek(2).kind == Token::Ident &&
            (peek(2).text == "layer" || peek(2).text == "model") && is_punct("(", 3)) {
            auto st = std::make_shared<Stmt>();
            st->kind = Stmt::Block;
            st->at = peek().at;
            st->block_name = next().text;
            next();  // '='
            st->block_kind = next().text;
            expect("(");
            if (!is_punct(")")) {
                st->params.push_back(ident());
                while (is_punct(",")) {
                    next();
                    st->params.push_back(ident());
                }
            }
            expect(")");
            expect("{");
            st->body = statements(true);
            expect("}");
            if (is_punct(";")) next();
            return st;
        }
        auto st = std::make_shared<Stmt>();
        st->at = peek().at;
        ExprP e = expr();
        if (is_punct("=")) {
            next();
            if (e->path().empty()) throw DslError(e->at, "cannot assign to this expression");
            st->kind = Stmt::Assign;
            st->target = e;
            st->value = expr();
        } else {
            st->kind = Stmt::Eval;
            st->value = e;
        }
        expect(";");
        return st;
    }

    ExprP binary(const std::string &op, ExprP l, ExprP r, SrcLoc at) {
        auto e = std::make_shared<Expr>();
        e->kind = Expr::Binary;
        e->name = op;
        e->lhs = std::move(l);
        e->rhs = std::move(r);
        e->at = at;
        return e;
    }

    ExprP expr() {
        ExprP l = term();
        while (is_punct("+") || is_punct("-")) {
            const Token op = next();
            l = binary(op.text, l, term(), op.at);
        }
        return l;
    }
    ExprP term() {
        ExprP l = unary();
        while (is_punct("*") || is_punct("/")) {
            const Token op = next();
            l = binary(op.text, l, unary(), op.at);
        }
        return l;
    }
    ExprP unary() {
        if (is_punct("-")) {
            const Token op = next();
            ExprP v = unary();
            if (v->kind == Expr::Number) {
                v->num = -v->num;
                v->at = op.at;
                return v;
            }
            auto e = std::make_shared<Expr>();
            e->kind = Expr::Neg;
            e->obj = v;
            e->at = op.at;
            return e;
        }
        return postfix();
    }
    ExprP postfix() {
        ExprP e = primary();
        while (true) {
            if (is_punct(".")) {
                const Token dot = next();
                auto m = std::make_shared<Expr>();
                m->kind = Expr::Member;
                m->obj = e;
                m->name = ident();
                m->at = dot.at;
                e = m;
            } else if (is_punct("(")) {
                const Token lp = next();
                auto c = std::make_shared<Expr>();
                c->kind = Expr::Call;
                c->obj = e;
                c->at = e->at;
                if (!is_punct(")")) {
                    while (true) {
                        std::string kw;
                        if (peek().kind == Token::Ident && is_punct("=", 1)) {
                            kw = next().text;
                            next();
                        }
                        c->kw.push_back(kw);
                        c->args.push_back(expr());
                        if (!is_punct(",")) break;
                        next();
                    }
                }
                expect(")");
                (void)lp;
                e = c;
            } else {
                return e;
            }
        }
    }
    ExprP primary() {
        const Token t = next();
        auto e = std::make_shared<Expr>();
        e->at = t.at;
        switch (t.kind) {
        case Token::Ident:
            if (t.text == "true" || t.text == "false") {
                e->kind = Expr::Bool;
                e->bval = t.text == "true";
            } else if (t.text == "null") {
                e->kind = Expr::Null;
            } else {
                e->kind = Expr::Ident;
                e->name = t.text;
            }
            return e;
        case Token::Number:
            e->kind = Expr::Number;
            e->num = std::stod(t.text);
            e->is_int = t.text.find_first_of(".eE") == std::string::npos;
            return e;
        case Token::String:
            e->kind = Expr::String;
            e->name = t.text;
            return e;
        case Token::Punct:
            if (t.text == "(") {
                ExprP inner = expr();
                expect(")");
                return inner;
            }
            throw DslError(t.at, "unexpected '" + t.text + "'");
        case Token::End:
            throw DslError(t.at, "unexpected end of file");
        }
        throw DslError(t.at, "unexpected token");
    }
};

}  // namespace

Program parse_program(const std::string &text, const std::string &source_name) {
    Parser ps(lex(text));
    Program prog;
    prog.source_name = source_name;
    prog.stmts = ps.statements(false);
    return prog;
}

Program parse_file(const std::string &path) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open DSL file " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse_program(ss.str(), path);
}

}  // namespace galac
