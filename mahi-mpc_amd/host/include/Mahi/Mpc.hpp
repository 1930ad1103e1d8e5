#pragma once
#include <Mahi/Mpc/External.hpp>
#include <Mahi/Mpc/BatchModelControl.hpp>
#include <Mahi/Mpc/ModelControl.hpp>
#include <Mahi/Mpc/ModelGenerator.hpp>
#include <Mahi/Mpc/ModelParameters.hpp>
