// SDL front end: a C++ restatement of raysnail's POV-Ray-like scene parser (src/sdl_parser.rs).
//
// The reference parser is a token-level recursive descent whose quirks decide what a file means
// (silent `expect` failures, the token skipped after a #declare'd or #while'd expression, `-` as a
// token separator, loops replayed by rewinding the token cursor), so this file keeps the same token
// stream and the same accept / expect decisions:
//   tokenizer          sdl_parser.rs:261-327 (split_inclusive on the separator set, trim, `//` comments)
//   statement list     :347-441 (first matching statement parser wins; an invalid statement = parse error)
//   objects            :444-812 (camera, light, sphere, box, quadric, object, difference, intersection)
//   directives         :815-933 (#declare, #while, #end)
//   modifiers/texture  :946-1098 (translate / rotate (degrees -> radians, x then y then z) / scale,
//                                 pigment color|checker, finish reflection|phong|phong_size, surface)
//   expressions        :1271-1401 (unary minus on the first term, + - * / left to right, parentheses,
//                                 #declare'd floats, Rust f64 literals)
// Where the reference panics (`unwrap` on a missing vector or float) the parser throws
// raysnail::Error; an invalid statement gives Error("Parse error") like SdlParser::parse's Err.
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <unordered_map>
#include <variant>
#include <vector>

#include "raysnail.hpp"

namespace raysnail {
namespace {

enum class Sym {
    Camera, Location, LookAt, Sphere, Box, Quadric, Light, Intersection, Difference, Object,
    Plus, Minus, Multiply, Divide, Equal, BlockOpen, BlockClose, VectorOpen, VectorClose, ParenOpen,
    ParenClose, Comma, Semicolon, Translate, Rotate, Scale, Texture, Pigment, Finish, Surface, Metallic,
    Reflection, Color, Rgb, Angle, Diffuse, Phong, PhongSize, Checker, Declare, While, End, Id, Eof, None
};

const std::unordered_map<std::string, Sym>& keywords() {  // build_symbol_map, sdl_parser.rs:207-258
    static const std::unordered_map<std::string, Sym> m = {
        {"camera", Sym::Camera}, {"look_at", Sym::LookAt}, {"location", Sym::Location},
        {"{", Sym::BlockOpen}, {"}", Sym::BlockClose}, {"intersection", Sym::Intersection},
        {"difference", Sym::Difference}, {"object", Sym::Object}, {"<", Sym::VectorOpen},
        {">", Sym::VectorClose}, {",", Sym::Comma}, {";", Sym::Semicolon}, {"sphere", Sym::Sphere},
        {"box", Sym::Box}, {"quadric", Sym::Quadric}, {"light", Sym::Light}, {"texture", Sym::Texture},
        {"pigment", Sym::Pigment}, {"finish", Sym::Finish}, {"surface", Sym::Surface},
        {"reflection", Sym::Reflection}, {"metallic", Sym::Metallic}, {"color", Sym::Color},
        {"rgb", Sym::Rgb}, {"checker", Sym::Checker}, {"angle", Sym::Angle}, {"diffuse", Sym::Diffuse},
        {"phong", Sym::Phong}, {"phong_size", Sym::PhongSize}, {"translate", Sym::Translate},
        {"rotate", Sym::Rotate}, {"scale", Sym::Scale}, {"+", Sym::Plus}, {"-", Sym::Minus},
        {"*", Sym::Multiply}, {"/", Sym::Divide}, {"(", Sym::ParenOpen}, {")", Sym::ParenClose},
        {"=", Sym::Equal}, {"#declare", Sym::Declare}, {"#while", Sym::While}, {"#end", Sym::End},
    };
    return m;
}

bool is_separator(char c) {
    switch (c) {
    case ' ': case ',': case ';': case '(': case ')': case '<': case '>': case '{': case '}':
    case '+': case '-': case '*': case '/': case '\n': return true;
    default: return false;
    }
}

// str::trim: strip leading / trailing whitespace
std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

struct Token {
    std::string text;
    uint32_t line;
};

void tokenize_line(const std::string& raw, uint32_t line_no, std::vector<Token>& out) {
    const size_t cut = raw.find("//");  // strip_line_comments: the part before the first "//"
    const std::string line = cut == std::string::npos ? raw : raw.substr(0, cut);
    auto push = [&](const std::string& piece) {
        std::string t = trim(piece);
        if (!t.empty()) out.push_back({t, line_no});
    };
    size_t start = 0;
    for (size_t i = 0; i < line.size(); ++i) {
        if (is_separator(line[i])) {  // a piece ending in a separator: the text before it, then it
            push(line.substr(start, i - start));
            push(std::string(1, line[i]));
            start = i + 1;
        }
    }
    if (start < line.size()) push(line.substr(start));
}

// Rust's `str::parse::<f64>` grammar on a token that contains no separator (so no sign):
// digits [. digits] [e digits] | . digits [e digits] | inf | infinity | nan (case-insensitive).
bool parse_rust_f64(const std::string& s, double& v) {
    std::string low;
    for (char c : s) low.push_back((char)std::tolower((unsigned char)c));
    if (low == "inf" || low == "infinity") { v = INFINITY; return true; }
    if (low == "nan") { v = NAN; return true; }
    size_t i = 0, n = s.size();
    size_t int_digits = 0, frac_digits = 0;
    while (i < n && std::isdigit((unsigned char)s[i])) { ++i; ++int_digits; }
    if (i < n && s[i] == '.') {
        ++i;
        while (i < n && std::isdigit((unsigned char)s[i])) { ++i; ++frac_digits; }
    }
    if (int_digits + frac_digits == 0) return false;
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        size_t exp_digits = 0;
        while (i < n && std::isdigit((unsigned char)s[i])) { ++i; ++exp_digits; }
        if (exp_digits == 0) return false;
    }
    if (i != n) return false;
    v = std::strtod(s.c_str(), nullptr);  // correctly rounded, like Rust's parser
    return true;
}

struct Invalid {};
struct Directive {};
using Entity = std::variant<Invalid, Directive, CameraData, LightData, HittableRef, double, Vec3>;

class Parser {
public:
    explicit Parser(std::vector<Token> toks) : tokens_(std::move(toks)) {}

    bool parse_root(SceneData& scene) {  // :336-341
        nextsym();
        while (pos_ < tokens_.size()) {  // parse_statement_list, :344-379
            Entity e = statement();
            if (std::holds_alternative<HittableRef>(e)) scene.hittables.add(std::get<HittableRef>(e));
            else if (std::holds_alternative<LightData>(e)) scene.lights.push_back(std::get<LightData>(e));
            else if (std::holds_alternative<CameraData>(e)) scene.camera = std::get<CameraData>(e);
            else if (std::holds_alternative<Invalid>(e)) return false;
        }
        return true;
    }

private:
    std::vector<Token> tokens_;
    size_t pos_ = 0;
    Sym sym_ = Sym::None;
    std::map<std::string, Entity> declares_;
    std::vector<size_t> loops_;

    const std::string& text() const { return pos_ < tokens_.size() ? tokens_[pos_].text : tokens_.back().text; }
    uint32_t line() const { return pos_ < tokens_.size() ? tokens_[pos_].line : (uint32_t)tokens_.size(); }

    [[noreturn]] void fail(const char* what) const {
        std::ostringstream os;
        os << "SDL line " << line() << ": " << what << ", found '" << text() << "'";
        throw Error(RS_E_INVALID, os.str());
    }

    void nextsym() {
        ++pos_;
        if (pos_ < tokens_.size()) {
            auto it = keywords().find(tokens_[pos_].text);
            sym_ = it == keywords().end() ? Sym::Id : it->second;
        } else {
            sym_ = Sym::Eof;
        }
    }
    bool accept(Sym s) {  // accept / expect / expect_quiet are the same test upstream
        if (sym_ != s) return false;
        nextsym();
        return true;
    }

    // ---- statements (:382-441): the first parser that recognises its keyword wins
    Entity statement() {
        Entity e;
        if (!std::holds_alternative<Invalid>(e = camera())) return e;
        if (!std::holds_alternative<Invalid>(e = light())) return e;
        if (!std::holds_alternative<Invalid>(e = sphere())) return e;
        if (!std::holds_alternative<Invalid>(e = box())) return e;
        if (!std::holds_alternative<Invalid>(e = quadric())) return e;
        if (!std::holds_alternative<Invalid>(e = object())) return e;
        if (!std::holds_alternative<Invalid>(e = csg(Sym::Difference))) return e;
        if (!std::holds_alternative<Invalid>(e = csg(Sym::Intersection))) return e;
        if (!std::holds_alternative<Invalid>(e = declare())) return e;
        if (!std::holds_alternative<Invalid>(e = while_())) return e;
        if (!std::holds_alternative<Invalid>(e = end_())) return e;
        return Invalid{};
    }

    Entity camera() {  // :444-477, items :519-541
        if (!accept(Sym::Camera)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        CameraData cam;
        while (sym_ != Sym::BlockClose) {
            if (sym_ == Sym::Location) { nextsym(); cam.location = need_vector(); }
            else if (sym_ == Sym::LookAt) { nextsym(); cam.look_at = need_vector(); }
            else if (sym_ == Sym::Angle) { nextsym(); cam.fov_angle = need_expression(); }
            else return Invalid{};
        }
        nextsym();
        return cam;
    }

    Entity light() {  // :480-516
        if (!accept(Sym::Light)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        LightData l;
        std::optional<Vec3> loc = vector();
        if (!loc) return Invalid{};
        accept(Sym::Comma);
        std::optional<Color> col = color();
        if (!col) return Invalid{};
        accept(Sym::BlockClose);
        l.location = *loc;
        l.color = *col;
        return l;
    }

    Entity sphere() {  // :543-574
        if (!accept(Sym::Sphere)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        const Vec3 c = need_vector();
        accept(Sym::Comma);
        const double r = need_expression();
        MaterialRef mat = texture();
        TransformStack st = modifiers();
        accept(Sym::BlockClose);
        return facade(st, std::make_shared<Sphere>(c, r, mat));
    }

    Entity box() {  // :577-603
        if (!accept(Sym::Box)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        const Vec3 a = need_vector();
        accept(Sym::Comma);
        const Vec3 b = need_vector();
        MaterialRef mat = texture();
        TransformStack st = modifiers();
        accept(Sym::BlockClose);
        return facade(st, std::make_shared<Box>(a, b, mat));
    }

    Entity quadric() {  // :606-639; POV <A,B,C>,<D,E,F>,<G,H,I>,J -> Quadric::new(A, D, E, G, B, F, H, C, I, J)
        if (!accept(Sym::Quadric)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        const Vec3 v1 = need_vector();
        accept(Sym::Comma);
        const Vec3 v2 = need_vector();
        accept(Sym::Comma);
        const Vec3 v3 = need_vector();
        accept(Sym::Comma);
        const double j = need_expression();
        MaterialRef mat = texture();
        TransformStack st = modifiers();
        auto q = std::make_shared<Quadric>(v1.x, v2.x, v2.y, v3.x, v1.y, v2.z, v3.y, v1.z, v3.z, j, mat);
        accept(Sym::BlockClose);
        return facade(st, q);
    }

    Entity object() {  // :642-682: a #declare'd hittable, shared, under new modifiers
        if (!accept(Sym::Object)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        const std::string ident = identifier();
        TransformStack st = modifiers();
        accept(Sym::BlockClose);
        auto it = declares_.find(ident);
        if (it == declares_.end()) fail("undeclared identifier in object");  // entity.unwrap() panics
        if (!std::holds_alternative<HittableRef>(it->second)) return Invalid{};
        return facade(st, std::get<HittableRef>(it->second));
    }

    Entity csg(Sym kind) {  // difference :685-730, intersection :733-777
        if (!accept(kind)) return Invalid{};
        if (!accept(Sym::BlockOpen)) return Invalid{};
        Entity e1 = statement();
        if (!std::holds_alternative<HittableRef>(e1)) return Invalid{};
        Entity e2 = statement();
        if (!std::holds_alternative<HittableRef>(e2)) return Invalid{};
        MaterialRef mat = texture();
        TransformStack st = modifiers();
        HittableRef o;
        if (kind == Sym::Difference)
            o = std::make_shared<Difference>(std::get<HittableRef>(e1), std::get<HittableRef>(e2), mat);
        else
            o = std::make_shared<Intersection>(std::get<HittableRef>(e1), std::get<HittableRef>(e2), mat);
        accept(Sym::BlockClose);
        return facade(st, o);
    }

    Entity declare() {  // :780-820
        if (!accept(Sym::Declare)) return Invalid{};
        const std::string ident = identifier();
        if (!accept(Sym::Equal)) return Invalid{};
        if (std::optional<double> v = expression()) {
            nextsym();              // skips the token after the expression (the ';')
            accept(Sym::Semicolon);
            declares_[ident] = *v;
            return Directive{};
        }
        if (std::optional<Vec3> v = vector()) {
            accept(Sym::Semicolon);
            declares_[ident] = *v;
            return Directive{};
        }
        declares_[ident] = statement();   // stored even when invalid
        return Directive{};
    }

    Entity while_() {  // :823-863
        const size_t loop_start = pos_;
        if (!accept(Sym::While)) return Invalid{};
        if (!accept(Sym::ParenOpen)) return Invalid{};
        std::optional<double> v1 = expression();
        if (!v1) return Invalid{};
        nextsym();                  // skips the '<'
        accept(Sym::VectorOpen);
        std::optional<double> v2 = expression();
        if (!v2) return Invalid{};
        nextsym();                  // skips the ')'
        if (*v1 < *v2) {
            loops_.push_back(loop_start);
        } else {
            while (sym_ != Sym::End) {  // fast_forward_to_end
                if (sym_ == Sym::Eof) fail("#while without #end");
                nextsym();
            }
            nextsym();
        }
        return Directive{};
    }

    Entity end_() {  // :875-889: rewind to the #while token
        if (!accept(Sym::End)) return Invalid{};
        if (loops_.empty()) fail("#end without #while");
        const size_t start = loops_.back();
        loops_.pop_back();
        pos_ = start - 1;
        nextsym();
        return Directive{};
    }

    // ---- pieces
    static HittableRef facade(const TransformStack& st, HittableRef o) {  // :892-899
        if (st.len() > 0) return std::make_shared<TfFacade>(std::move(o), st);
        return o;
    }

    // parse_translate / parse_rotate / parse_scale (:1167-1246): each consumes its keyword and
    // yields nothing when no operand follows, and the chain then tries the next modifier
    std::optional<Vec3> translate_() {
        if (accept(Sym::Translate)) return vector();
        return std::nullopt;
    }
    std::optional<Vec3> rotate_() {
        if (accept(Sym::Rotate)) return vector();
        return std::nullopt;
    }
    std::optional<Vec3> scale_() {
        if (!accept(Sym::Scale)) return std::nullopt;
        if (std::optional<Vec3> v = vector()) return v;
        if (std::optional<double> f = float_()) return Vec3{*f, *f, *f};
        return std::nullopt;
    }

    TransformStack modifiers() {  // :902-937; rotate: degrees -> radians, x then y then z
        TransformStack st;
        const double pi = 3.14159265358979323846;  // std::f64::consts::PI
        while (true) {
            if (std::optional<Vec3> v = translate_()) {
                st.push(Transform::translate(*v));
            } else if (std::optional<Vec3> r = rotate_()) {
                if (r->x != 0.0) st.push(Transform::rotate_by_x_axis(r->x * pi / 180.0));
                if (r->y != 0.0) st.push(Transform::rotate_by_y_axis(r->y * pi / 180.0));
                if (r->z != 0.0) st.push(Transform::rotate_by_z_axis(r->z * pi / 180.0));
            } else if (std::optional<Vec3> sc = scale_()) {
                st.push(Transform::scale(*sc));
            } else {
                break;
            }
        }
        return st;
    }

    MaterialRef texture() {  // :939-966; no texture block -> None (the world default material)
        if (!accept(Sym::Texture)) return nullptr;
        if (!accept(Sym::BlockOpen)) return nullptr;
        std::optional<Texture> tex = pigment();
        MaterialRef mat = finish(tex ? *tex : Texture::color(Color{1.f, 1.f, 1.f, 1.f}));
        accept(Sym::BlockClose);
        return mat;
    }

    std::optional<Texture> pigment() {  // :968-986; checker scale 2.0
        if (!accept(Sym::Pigment)) return std::nullopt;
        if (!accept(Sym::BlockOpen)) return std::nullopt;
        if (std::optional<Color> c = color()) {
            accept(Sym::Rgb);
            accept(Sym::BlockClose);
            return Texture::color(*c);
        }
        if (accept(Sym::Checker)) {  // parse_checker, :1133-1154
            std::optional<Color> c1 = color();
            if (!c1) return std::nullopt;
            accept(Sym::Comma);
            std::optional<Color> c2 = color();
            if (!c2) return std::nullopt;
            accept(Sym::BlockClose);
            return Texture::checker(*c1, *c2, 2.0);
        }
        return std::nullopt;
    }

    static CommonMaterialSettings settings(double phong, double phong_size) {  // :1091-1100
        CommonMaterialSettings s;
        if (phong > 0.0) {
            s.phong_factor = phong * 4.0;
            s.phong_exponent = (int32_t)(phong_size * 0.1);  // `as i32` truncates
        }
        return s;
    }

    MaterialRef finish(const Texture& tex) {  // :989-1089
        if (accept(Sym::Finish)) {
            if (!accept(Sym::BlockOpen)) return std::make_shared<Lambertian>(tex);
            double phong = 0.0, phong_size = 40.0, reflection = 0.0;
            while (true) {
                if (accept(Sym::Reflection)) reflection = need_float();
                else if (accept(Sym::Phong)) phong = need_float();
                else if (accept(Sym::PhongSize)) phong_size = need_float();
                else break;
            }
            accept(Sym::BlockClose);
            auto lam = std::make_shared<Lambertian>(tex);
            lam->set(settings(phong, phong_size));
            if (reflection == 0.0) return lam;
            auto metal = std::make_shared<Metal>(tex);
            metal->set(settings(phong, phong_size));
            return std::make_shared<MixedMaterial>(metal, lam, reflection);
        }
        if (accept(Sym::Surface)) {
            if (!accept(Sym::BlockOpen)) return std::make_shared<Lambertian>(tex);
            MaterialRef m;
            if (accept(Sym::Metallic)) {
                if (accept(Sym::Diffuse)) m = std::make_shared<DiffuseMetal>(need_float(), tex);
                else m = std::make_shared<Metal>(tex);
            } else {
                m = std::make_shared<Lambertian>(tex);
            }
            accept(Sym::BlockClose);
            return m;
        }
        return std::make_shared<Lambertian>(tex);  // Lambertian is the default
    }

    std::optional<Color> color() {  // :1249-1261: color [rgb] <r, g, b>, f64 -> f32
        if (!accept(Sym::Color)) return std::nullopt;
        accept(Sym::Rgb);
        std::optional<Vec3> v = vector();
        if (!v) return std::nullopt;
        return Color::new64(v->x, v->y, v->z, 1.0);
    }

    std::string identifier() {  // :1157-1164: the current token, whatever it is
        std::string id = text();
        nextsym();
        return id;
    }

    std::optional<Vec3> vector() {  // :1263-1283
        if (!accept(Sym::VectorOpen)) return std::nullopt;
        const double x = need_expression();
        accept(Sym::Comma);
        const double y = need_expression();
        accept(Sym::Comma);
        const double z = need_expression();
        accept(Sym::VectorClose);
        return Vec3{x, y, z};
    }
    Vec3 need_vector() {
        std::optional<Vec3> v = vector();
        if (!v) fail("expected a vector");
        return *v;
    }

    std::optional<double> expression() {  // :1286-1330
        double e;
        if (accept(Sym::Minus)) {
            std::optional<double> t = term();
            if (!t) return std::nullopt;
            e = -*t;
        } else {
            std::optional<double> t = term();
            if (!t) return std::nullopt;
            e = *t;
        }
        while (true) {
            if (accept(Sym::Minus)) {
                std::optional<double> t = term();
                if (!t) return std::nullopt;
                e -= *t;
            } else if (accept(Sym::Plus)) {
                std::optional<double> t = term();
                if (!t) return std::nullopt;
                e += *t;
            } else {
                break;
            }
        }
        return e;
    }
    double need_expression() {
        std::optional<double> v = expression();
        if (!v) fail("expected an expression");
        return *v;
    }

    std::optional<double> term() {  // :1333-1366
        std::optional<double> f = factor();
        if (!f) return std::nullopt;
        double v = *f;
        while (true) {
            if (accept(Sym::Multiply)) {
                std::optional<double> g = factor();
                if (!g) return std::nullopt;
                v *= *g;
            } else if (accept(Sym::Divide)) {
                std::optional<double> g = factor();
                if (!g) return std::nullopt;
                v /= *g;
            } else {
                break;
            }
        }
        return v;
    }

    std::optional<double> factor() {  // :1369-1396
        if (accept(Sym::ParenOpen)) {
            std::optional<double> e = expression();
            if (accept(Sym::ParenClose)) return e;
            return std::nullopt;
        }
        auto it = declares_.find(text());
        if (it != declares_.end() && std::holds_alternative<double>(it->second)) {
            const double v = std::get<double>(it->second);
            nextsym();
            return v;
        }
        return float_();
    }

    std::optional<double> float_() {  // :1399-1411
        double v;
        if (!parse_rust_f64(text(), v)) return std::nullopt;
        nextsym();
        return v;
    }
    double need_float() {
        std::optional<double> v = float_();
        if (!v) fail("expected a number");
        return *v;
    }
};

std::vector<Token> tokens_of(const std::string& text) {  // read_tokens, :304-327
    std::vector<Token> toks;
    toks.push_back({"START", 0});  // fills the unused position 0
    std::istringstream in(text);
    std::string line;
    uint32_t n = 1;
    while (std::getline(in, line)) {  // str::lines: "\n" or "\r\n" endings
        if (!line.empty() && line.back() == '\r') line.pop_back();
        tokenize_line(line, n, toks);
        ++n;
    }
    return toks;
}

}  // namespace

SceneData SdlParser::parse_text(const std::string& text) {
    SceneData scene;
    Parser p(tokens_of(text));
    if (!p.parse_root(scene)) throw Error(RS_E_INVALID, "Parse error");
    return scene;
}

SceneData SdlParser::parse(const std::string& filename) {
    std::ifstream f(filename, std::ios::binary);
    if (!f) throw Error(RS_E_INVALID, "cannot read " + filename);  // read_to_string(..).unwrap() panics
    std::ostringstream ss;
    ss << f.rdbuf();
    return parse_text(ss.str());
}

}  // namespace raysnail
