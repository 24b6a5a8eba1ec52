// Config files (reference src/config.cc semantics over addapt/yaml.hh).
#include "addapt/config.hh"

#include <regex>

#include "addapt/yaml.hh"

namespace addapt {

namespace {

// config.cc:23-48: a section may appear in only one of the files
yaml::Node find_section(const std::vector<string> &files, const string &name, bool required = true) {
    yaml::Node section;
    bool found = false;
    for (auto &f : files) {
        yaml::Node doc = yaml::load_file(f);
        const yaml::Node &s = doc[name];
        if (s) {
            if (found) throw string("found 2 '" + name + "' configurations");
            section = s;
            found = true;
        }
    }
    if (!found && required) throw string("no '" + name + "' configuration");
    return section;
}

}  // namespace

DevicePtr device_from_yaml(std::vector<string> files) {
    auto device = std::make_shared<Device>(find_section(files, "sequence").as_string());
    yaml::Node macro = find_section(files, "macrostates");
    for (auto &kv : macro.map) device->add_macrostate(kv.first, kv.second.as_string());
    return device;
}

ScoreFunctionPtr scorefxn_from_yaml(std::vector<string> files) {
    auto sf = std::make_shared<ScoreFunction>();
    yaml::Node obj = find_section(files, "objective");
    *sf += score_term_from_str(ConditionEnum::APO, obj["apo"].as_string());
    *sf += score_term_from_str(ConditionEnum::HOLO, obj["holo"].as_string());
    yaml::Node apt = find_section(files, "aptamer");
    sf->aptamer(std::make_shared<Aptamer>(apt["sequence"].as_string(), apt["fold"].as_string(),
                                          std::stod(apt["affinity"].as_string())));
    yaml::Node ctx = find_section(files, "contexts", false);
    for (auto &kv : ctx.map)
        sf->add_context(kv.first, std::make_shared<Context>(kv.second[0].as_string(), kv.second[1].as_string()));
    return sf;
}

ScoreTermPtr score_term_from_str(ConditionEnum condition, string spec) {
    static const std::regex pattern("(not )?(\\w+)");
    std::smatch m;
    if (std::regex_match(spec, m, pattern))
        return std::make_shared<MacrostateProbTerm>(m[2], condition,
                                                    m[1].matched ? FavorableEnum::NO : FavorableEnum::YES);
    throw string("can't understand objective: '" + spec + "'");
}

ThermostatPtr thermostat_from_yaml(std::vector<string> files) {
    yaml::Node s = find_section(files, "thermostat", false);
    return thermostat_from_str(s ? s.as_string() : "1");
}

// "5" | "5 to 0 in 300 steps" | "auto [rate% [period [T0]]]" (config.cc:113-175)
ThermostatPtr thermostat_from_str(string spec) {
    static const std::regex fixed("([0-9.e+-]+)");
    static const std::regex anneal("([0-9.e+-]+) to ([0-9.e+-]+) in ([0-9]+) steps");
    static const std::regex autos("auto(?:\\s+([0-9.]+)%(?:\\s+([0-9]+)(?:\\s+([0-9.e+-]+))?)?)?");
    std::smatch m;
    if (std::regex_match(spec, m, fixed)) return std::make_shared<FixedThermostat>(std::stod(m[1]));
    if (std::regex_match(spec, m, anneal))
        return std::make_shared<AnnealingThermostat>(std::stoi(m[3]), std::stod(m[1]), std::stod(m[2]));
    if (std::regex_match(spec, m, autos)) {
        const double rate = std::stod(m[1].length() ? m[1].str() : "50") / 100;
        const int period = int(std::stod(m[2].length() ? m[2].str() : "100"));
        const double t0 = std::stod(m[3].length() ? m[3].str() : "1");
        return std::make_shared<AutoScalingThermostat>(rate, unsigned(period), t0);
    }
    throw string("can't make a thermostat from '" + spec + "'");
}

}  // namespace addapt
